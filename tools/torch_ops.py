"""The torch (non-library) device ops of one bench training step, with the Python line that
issued each: what the graph replays besides the library's kernels (copies, fills, elementwise).

    python tools/torch_ops.py [--global-batch 512]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse_args(sys.argv[1:] + ["--no-cpu-baseline", "--no-secondary"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ts = bench.TrainStep(a, "c4", 0, 1, dev)
    for _ in range(3):
        ts.eager_step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        ts.eager_step()
        torch.cuda.synchronize()
    # aten ops with device time, grouped by the innermost frame inside this repo
    rows = {}
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        if ev.device_time_total <= 0:
            continue
        if any(c.name.startswith("aten::") and c.device_time_total > 0 for c in ev.cpu_children):
            continue   # count the innermost aten op only
        where = "?"
        for fr in (ev.stack or []):
            if "/repo/" in fr or "sp-nerf_amd" in fr or "bench.py" in fr:
                where = fr.split("/")[-1]
                break
        k = (ev.name, where)
        n, t = rows.get(k, (0, 0.0))
        rows[k] = (n + 1, t + ev.device_time_total)
    tot = 0.0
    for (name, where), (n, t) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:9.1f} us {n:3d}x {name:28s} {where}")
        tot += t
    print(f"total {tot:.1f} us of torch device ops per eager step (batch {ts.B})")
    ts.close()


if __name__ == "__main__":
    main()
