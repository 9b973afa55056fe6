"""Training-trajectory spread vs precision (tools only): several arms trained side by side with
the C3 flags on the real JAX_269 targets (bench.psnr_long's setup), same batches and on-device
draws; an arm = (name, MLP precision, relative init perturbation, Philox seed).  Prints the
held-out PSNR of each arm — an fp32 arm with a 1e-6 init perturbation shows how far two runs of
the SAME arithmetic drift apart, the yardstick for the bf16-vs-fp32 gap.
    python tools/psnr_arms.py --steps 300 --batch 256"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import spnerf_amd  # noqa: E402
from spnerf_amd import PhiloxRandom, random_source  # noqa: E402
from spnerf_amd.losses import FusedRenderLoss  # noqa: E402
from spnerf_amd.scene import synthetic_scene  # noqa: E402

# (name, precision, init perturbation, Philox seed, option emu_bf16: the fp32 MLP with bf16 rounding of
# 4 = its GEMM weights, 1 = forward activations, 2 = backward dX)
ARMS = [("fp32", "fp32", 0.0, 3, 0), ("fp32_perturbed", "fp32", 1e-6, 3, 0), ("bf16", "bf16", 0.0, 3, 0),
        ("bf16_perturbed", "bf16", 1e-6, 3, 0), ("fp32_other_draws", "fp32", 0.0, 4, 0),
        ("fp32_emu_w", "fp32", 0.0, 3, 4), ("fp32_emu_fwd", "fp32", 0.0, 3, 1), ("fp32_emu_bwd", "fp32", 0.0, 3, 2),
        ("fp32_emu_all", "fp32", 0.0, 3, 7)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--n-eval", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--arms", default=",".join(a[0] for a in ARMS))
    ap.add_argument("--seeds", default="", help="replica study: e.g. 3,4,5 -> each of --kinds per seed "
                    "(init perturbed 1e-6 with that seed unless it is the first, Philox seed = it)")
    ap.add_argument("--kinds", default="fp32,bf16", help="with --seeds: fp32, bf16, emu (fp32 + emu_bf16 7)")
    a = ap.parse_args()
    if a.seeds:
        seeds = [int(x) for x in a.seeds.split(",")]
        kinds = {"fp32": ("fp32", 0), "bf16": ("bf16", 0), "emu": ("fp32", 7)}
        arms = [(f"{k}_s{sd}", kinds[k][0], 0.0 if sd == seeds[0] else 1e-6, sd, kinds[k][1])
                for sd in seeds for k in a.kinds.split(",")]
    else:
        arms = [x for x in ARMS if x[0] in a.arms.split(",")]
    dev = "cuda:0"
    c = bench.CONFIGS["c3"]
    args = bench.make_args(c)
    R = synthetic_scene(4.0, seed=0, device=dev)
    rng = np.random.default_rng(3)
    perm = rng.permutation(R.rays.shape[0])
    held, pool = torch.as_tensor(perm[:a.n_eval], device=dev), perm[a.n_eval:]
    models, opts, srcs, emu = {}, {}, {}, {}
    for name, prec, eps, seed, e in arms:
        emu[name] = e
        torch.manual_seed(3)
        m = spnerf_amd.SPNeRF(num_sem_classes=3, s_embedding_factor=1, layers=8, feat=512, mapping=True, sem=True,
                              precision=prec).to(dev).use_flat_grads()
        if eps:
            g = torch.Generator(device="cpu").manual_seed(99 + seed)
            with torch.no_grad():
                for p in m.parameters():
                    p.mul_(1 + eps * torch.randn(p.shape, generator=g).to(dev))
        models[name], opts[name], srcs[name] = m, spnerf_amd.optim.Adam(list(m.parameters()), lr=a.lr), PhiloxRandom(seed)
    floss = FusedRenderLoss(c["sc_lambda"], 1.0, 1.0)

    def evaluate():
        out = {}
        for name, *_ in arms:
            spnerf_amd._lib.set_option("emu_bf16", emu[name])
            rgb = []
            with torch.no_grad(), random_source(PhiloxRandom(seed=1000)):
                for i0 in range(0, a.n_eval, 2048):
                    ii = held[i0:i0 + 2048]
                    rgb.append(spnerf_amd.render_rays({"coarse": models[name]}, args, R.rays[ii], None,
                                                      semantics=R.sems[ii], mode="test")["rgb_coarse"])
            out[name] = round(float(-10 * np.log10(float(torch.mean((torch.cat(rgb) - R.rgbs[held]) ** 2)))), 4)
        return out

    t0 = time.perf_counter()
    for step in range(a.steps):
        idx = torch.as_tensor(rng.choice(pool, a.batch, replace=False), device=dev)
        for name, *_ in arms:
            spnerf_amd._lib.set_option("emu_bf16", emu[name])
            opts[name].zero_grad(set_to_none=True)
            with random_source(srcs[name]):
                res = spnerf_amd.render_rays({"coarse": models[name]}, args, R.rays[idx], None, semantics=R.sems[idx],
                                             mode="train", valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                             target_std=R.depth_std[idx])
            loss, _ = floss(res, R.rgbs[idx], R.depths[idx], R.valid_depth[idx], R.depth_std[idx], R.sems[idx])
            loss.backward()
            opts[name].step()
        if (step + 1) % max(1, a.steps // 5) == 0:
            print(json.dumps({"step": step + 1, "seconds": round(time.perf_counter() - t0, 1), "psnr": evaluate()}),
                  flush=True)


if __name__ == "__main__":
    main()
