"""spnerf_amd.optim.Adam (spnerf_adam_step, one launch for the parameter list) vs torch.optim.Adam
(single-tensor loop, reference main.py's optimizer) — needs an MI355X.

Same update formula; the two differ only in fp32 rounding order inside a step, so parameters
after several steps agree to a few ulp (held at 1e-6 relative to the parameter scale).
"""
import pytest
import torch

import spnerf_amd.optim as sopt

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_adam_matches_torch():
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = [(512, 576), (512,), (3, 256), (1,), (7, 5), (4096 + 3,), (0,), (256, 3)]
    init = [torch.randn(s, generator=g) for s in shapes]
    a = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    b = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    oa = sopt.Adam(a, lr=5e-4)
    ob = torch.optim.Adam(b, lr=5e-4, foreach=False, fused=False)
    for it in range(6):
        grads = [torch.randn(s, generator=g).to(DEV) * (10.0 ** (it % 3 - 1)) for s in shapes]
        for p, q, gr in zip(a, b, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for p, q in zip(a, b):
        if p.numel() == 0:
            continue
        err = (p - q).abs().max().item()
        assert err <= 1e-6 * max(1.0, q.abs().max().item()), err
        st_a, st_b = oa.state[p], ob.state[q]
        for k in ("exp_avg", "exp_avg_sq"):  # a few ulp of the state's scale
            d = (st_a[k] - st_b[k]).abs().max().item()
            assert d <= 1e-6 * st_b[k].abs().max().item(), (k, d)
        assert int(st_a["step"]) == 6
