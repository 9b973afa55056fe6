"""Which torch ops launch the small non-library kernels of a C4 training step (fills, copies, adds):
one eager step of the bench's TrainStep under torch.profiler, the aten ops that ran device kernels
other than the library's, with their shapes and the autograd node (or Python frame) they ran under.
    python tools/fill_probe.py [--global-batch 512]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--global-batch", type=int, default=512)
cli = p.parse_args()
a = bench.parse_args(["--config", "c4", "--global-batch", str(cli.global_batch), "--no-cpu-baseline", "--no-secondary"])
dev = torch.device("cuda:0")
ts = bench.TrainStep(a, "c4", 0, 1, dev)
for _ in range(2):
    ts.eager_step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    ts.eager_step()
    torch.cuda.synchronize()
keep = ("fill", "zero", "ones", "copy", "add", "clone", "index", "cat", "mul", "to", "contiguous")
for e in prof.events():
    if e.device_type != torch.autograd.DeviceType.CPU or not e.name.startswith("aten::"):
        continue
    if not any(k in e.name for k in keep):
        continue
    kern = [k.name for k in e.kernels] if hasattr(e, "kernels") else []
    if not kern and getattr(e, "device_time_total", 0) == 0:
        continue
    stack = [s for s in (e.stack or []) if "spnerf_amd" in s or "bench.py" in s][:3]
    print(f"{e.name:28s} shapes={e.input_shapes} dev_us={getattr(e, 'device_time_total', 0):.1f} "
          f"kernels={[k[:40] for k in kern]} stack={stack}")
ts.close()
