"""bf16 MLP vs the reference fixtures, per output key and per gradient (tools only; the numbers
behind tests/test_gpu_bf16.py's per-key bounds).  Prints one JSON object per case.
    python tools/bf16_errors.py [case ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from test_gpu_parity import DEV, run_case  # noqa: E402


def main():
    cases = sys.argv[1:] or ["c1_w512", "c3_w512", "c3_w64", "beta_w64", "nomap_w64", "c3_test_w64", "c5_w512",
                             "fine_w64", "fine_sc_guided_w64"]
    for name in cases:
        data, res, params = run_case(name, "bf16")
        outs = {k[4:]: gu.rel_err(res[k[4:]].detach().cpu().numpy(), data[k]) for k in data if k.startswith("out_")}
        shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
        R = gu.projection_weights(shapes)
        loss = sum((res[k] * torch.tensor(R[k], device=DEV)).sum() for k in sorted(R))
        loss.backward()
        errs, sq_err, sq_ref = {}, 0.0, 0.0
        if any(k.startswith("grad_") for k in data):
            for n, p in params.items():
                ref = data["grad_" + n].astype(np.float64)
                g = p.grad.cpu().double().numpy() if p.grad is not None else np.zeros(tuple(p.shape))
                sq_err += float(np.sum((g - ref) ** 2))
                sq_ref += float(np.sum(ref ** 2))
                if ref.size >= 64 and np.any(ref):
                    errs[n] = gu.rel_err(g, ref)
        else:
            Q = gu.param_projections([(n, tuple(p.shape)) for n, p in params.items()])
            for n, p in params.items():
                proj = float((p.grad.double().cpu() * torch.tensor(Q[n]).double()).sum())
                gn = float(data["gnorm_" + n])
                sq_err += (proj - float(data["gproj_" + n])) ** 2
                sq_ref += gn ** 2
                if p.numel() >= 64 and gn > 0:
                    errs[n] = abs(proj - float(data["gproj_" + n])) / gn
        print(json.dumps({"case": name, "outputs": outs, "flat_grad": (sq_err / sq_ref) ** 0.5,
                          "worst_grads": dict(sorted(errs.items(), key=lambda kv: -kv[1])[:5])}), flush=True)


if __name__ == "__main__":
    main()
