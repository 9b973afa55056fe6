"""Which part of a training step breaks HIP-graph capture (diagnostic): capture render + loss +
backward with flat gradients, with and without gradient marks armed and deferred trunk
weight gradients.   python tools/capture_probe.py"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import spnerf_amd  # noqa: E402
from spnerf_amd import _lib  # noqa: E402
from spnerf_amd.losses import FusedRenderLoss  # noqa: E402
from spnerf_amd.scene import synthetic_scene  # noqa: E402


def run(marks, defer):
    dev = "cuda:0"
    R = synthetic_scene(4.0, seed=0, device=dev)
    idx = torch.arange(128, device=dev)
    torch.manual_seed(0)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True,
                          precision="bf16").to(dev).use_flat_grads()
    m.defer_trunk_wgrad = defer
    args = types.SimpleNamespace(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    floss = FusedRenderLoss(0.1, 1.0, 1.0)
    src = spnerf_amd.PhiloxRandom(seed=1)

    def step():
        res = spnerf_amd.render_rays({"coarse": m}, args, R.rays[idx], None, semantics=R.sems[idx], mode="train",
                                     valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                     target_std=R.depth_std[idx])
        loss, _ = floss(res, R.rgbs[idx], R.depths[idx], R.valid_depth[idx], R.depth_std[idx], R.sems[idx])
        loss.backward()

    _lib.grad_marks_arm(marks)
    try:
        with spnerf_amd.random_source(src):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            for p in m.parameters():
                p.grad = None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            g.replay()
            torch.cuda.synchronize()
        print(f"marks={marks} defer={defer}: capture + replay OK", flush=True)
    except Exception as e:
        print(f"marks={marks} defer={defer}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
    finally:
        _lib.grad_marks_arm(False)


if __name__ == "__main__":
    # one configuration per process (a failed capture can poison the context);
    # argv: marks defer [event-flags]
    if len(sys.argv) > 2:
        if len(sys.argv) > 3:
            _lib.set_option("grad_marks_flags", int(sys.argv[3]))
        run(sys.argv[1] == "1", sys.argv[2] == "1")
    else:
        import subprocess
        for cfg in (("0", "0"), ("0", "1"), ("1", "0", "2"), ("1", "0", "0"), ("1", "0", "1"), ("1", "0", "6")):
            subprocess.run([sys.executable, "-u", __file__, *cfg], check=False)
