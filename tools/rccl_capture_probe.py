"""RCCL inside a HIP-graph capture, rehearsed on ONE GPU (diagnostic; 2 ranks cannot share a
device under RCCL): a one-rank nccl process group, the C4-flags training step with its gradient
marks armed and dp.GradBuckets' overlapped all-reduces captured into the same graph, as bench.py
does at N > 1.  Checks that the capture succeeds and a replay's gradient equals the eager step's
bit for bit (one rank: the all-reduce is an identity).
    MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 python tools/rccl_capture_probe.py"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import spnerf_amd  # noqa: E402
from spnerf_amd import dp  # noqa: E402
from spnerf_amd.losses import FusedRenderLoss  # noqa: E402
from spnerf_amd.scene import synthetic_scene  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    R = synthetic_scene(4.0, seed=0, device=dev)
    idx = torch.arange(256, device=dev)
    torch.manual_seed(0)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True,
                          precision="bf16").to(dev).use_flat_grads()
    args = types.SimpleNamespace(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    floss = FusedRenderLoss(0.1, 1.0, 1.0)
    src = spnerf_amd.PhiloxRandom(seed=1)
    buckets = dp.GradBuckets(m, 1)
    buckets.arm(True)

    def step():
        res = spnerf_amd.render_rays({"coarse": m}, args, R.rays[idx], None, semantics=R.sems[idx], mode="train",
                                     valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                     target_std=R.depth_std[idx])
        loss, _ = floss(res, R.rgbs[idx], R.depths[idx], R.valid_depth[idx], R.depth_std[idx], R.sems[idx])
        loss.backward()
        buckets.launch(m._flat_grad, overlap=True, force=True)
        buckets.finish(m._flat_grad, force=True)

    def reset():
        for p in m.parameters():
            p.grad = None
        src.reset_step(-1)

    with spnerf_amd.random_source(src):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            reset()
            step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        eager = m._flat_grad.clone()
        reset()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        src.reset_step(-1)
        g.replay()
        torch.cuda.synchronize()
        same = torch.equal(eager, m._flat_grad)
    print(f"capture OK, {len(buckets.buckets)} buckets in the graph; replay == eager bitwise: {same}", flush=True)
    buckets.arm(False)
    dist.destroy_process_group()
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
