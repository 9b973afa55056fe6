"""Per-call timing of the MLP forward kernels on one MI355X (tools only).

    python tools/trunk_bench.py [--rays 1024] [--samples 128]

For a bf16 W=512 SPNeRF (semantic head on): forward with saved activations (training), without
(inference) and sigma-only, each with the fused trunk on and off; prints the library's
per-class HIP-event timings per forward call.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import spnerf_amd  # noqa: E402
from spnerf_amd import _lib  # noqa: E402
from spnerf_amd.spnerf import run_mlp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=1024)
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--modes", default="save,nosave,sigma")
    a = ap.parse_args()
    for o in a.option:
        k, v = o.split("=")
        _lib.set_option(k, int(v))
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    print("trunk2 resident workgroups per CU (save, inference):", _lib.lib().spnerf_debug_trunk2_occupancy(1),
          _lib.lib().spnerf_debug_trunk2_occupancy(0), flush=True)
    torch.manual_seed(0)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True, precision="bf16").to(dev)
    B, S = a.rays, a.samples
    rays = torch.zeros(B, 11, device=dev)
    rays[:, 0:3] = torch.rand(B, 3, device=dev) * 0.2 - 0.1
    d = torch.randn(B, 3, device=dev)
    rays[:, 3:6] = d / d.norm(dim=1, keepdim=True)
    rays[:, 7] = 1.0
    rays[:, 9] = 1.0
    z = torch.sort(torch.rand(B, S, device=dev), 1)[0].contiguous()
    lab = torch.randint(0, 3, (B,), device=dev)
    classes = ["trunk_bf16", "trunk_bf16_train", "heads_train", "gemm_nt_bf16", "gemm_nt_bf16d", "gemm_nt_f32", "heads_fwd",
               "heads_fused", "encode"]
    for mode in a.modes.split(","):
        for fused in ((1,) if a.option else (1, 0)):
            _lib.set_option("fused_trunk", fused)

            def call():
                if mode == "save":
                    return run_mlp(m, rays, z, 3, labels=lab)
                with torch.no_grad():
                    return run_mlp(m, rays, z, 3, labels=lab, sigma_only=mode == "sigma")
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            _lib.prof_reset()
            _lib.prof_enable(True)
            for _ in range(a.iters):
                out = call()
            torch.cuda.synchronize()
            _lib.prof_enable(False)
            res = {}
            for k in classes:
                r = _lib.prof_read(k)
                if r["launches"]:
                    res[k] = (r["launches"] // a.iters, round(1e3 * r["ms"] / a.iters, 1),
                              round(r["flop"] / (r["ms"] * 1e-3) / 1e12, 1) if r["flop"] else None)
            print(f"{mode:7s} fused={fused} P={B * S}: per call (launches, us, TF/s)", res, flush=True)
            del out
    _lib.set_option("fused_trunk", 1)


if __name__ == "__main__":
    main()
