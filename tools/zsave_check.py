"""bf16 gradient error against the reference fixtures with the library options given
(tools only): python tools/zsave_check.py c1_w512 zsave=0 zsave=1 "zsave=1 fused_trunk=0" """
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from spnerf_amd import _lib  # noqa: E402
from test_gpu_parity import DEV, run_case  # noqa: E402


def grad_err(name):
    data, res, params = run_case(name, "bf16")
    shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
    R = gu.projection_weights(shapes)
    loss = sum((res[k] * torch.tensor(R[k], device=DEV)).sum() for k in sorted(R))
    loss.backward()
    Q = gu.param_projections([(n, tuple(p.shape)) for n, p in params.items()])
    se = sr = 0.0
    per = {}
    for n, p in params.items():
        if "grad_" + n in data:
            ref = data["grad_" + n].astype(np.float64)
            g = p.grad.cpu().double().numpy() if p.grad is not None else np.zeros(tuple(p.shape))
            se += float(np.sum((g - ref) ** 2)); sr += float(np.sum(ref ** 2))
            per[n] = gu.rel_err(g, ref)
        else:
            proj = float((p.grad.double().cpu() * torch.tensor(Q[n]).double()).sum())
            gn = float(data["gnorm_" + n])
            se += (proj - float(data["gproj_" + n])) ** 2; sr += gn ** 2
            per[n] = abs(proj - float(data["gproj_" + n])) / max(gn, 1e-30)
    outs = {k[4:]: gu.rel_err(res[k[4:]].detach().cpu().numpy(), data[k]) for k in data if k.startswith("out_")}
    return (se / sr) ** 0.5, per, outs


name = sys.argv[1]
for spec in sys.argv[2:]:
    for kv in spec.split():
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    tot, per, outs = grad_err(name)
    worst = sorted(per.items(), key=lambda kv: -kv[1])[:5]
    print(f"{spec:28s} grad {tot:.3e}  worst {[(k, round(v, 4)) for k, v in worst]}")
    print(f"{'':28s} outs {max(outs.values()):.2e} {sorted(outs.items(), key=lambda kv: -kv[1])[:3]}", flush=True)


def grads(name, opts):
    for kv in opts.split():
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    data, res, params = run_case(name, "bf16")
    shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
    R = gu.projection_weights(shapes)
    loss = sum((res[k] * torch.tensor(R[k], device=DEV)).sum() for k in sorted(R))
    loss.backward()
    return {n: p.grad.detach().double().cpu().clone() for n, p in params.items() if p.grad is not None}


if os.environ.get("ZDIFF"):
    a = grads(name, "zsave=0")
    b = grads(name, "zsave=1")
    for n in a:
        print(f"{n:32s} |a| {a[n].norm():.3e} rel diff {(a[n] - b[n]).norm() / max(a[n].norm(), 1e-30):.3e}")
