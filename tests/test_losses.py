"""Training losses of the bench step vs the oracle restatement of modules/metrics.py (CPU)."""
import numpy as np
import torch

from oracle import ref_cpu
from spnerf_amd.losses import DepthLoss


def _inputs(B=257, S=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    z = torch.sort(torch.rand(B, S, generator=g), -1)[0]
    w = torch.rand(B, S, generator=g)
    w = w / w.sum(-1, keepdim=True)
    depth = (w * z).sum(-1).requires_grad_(True)
    res = {"z_vals_coarse": z, "weights_coarse": w, "depth_coarse": depth}
    td = torch.rand(B, generator=g)
    tw = torch.rand(B, generator=g)
    ts = 0.05 + 0.2 * torch.rand(B, generator=g)
    valid = (torch.rand(B, generator=g) < 0.68).long()
    return res, td, tw, valid, ts


def test_depth_loss_matches_reference_subset_form():
    for seed in range(4):
        res, td, tw, valid, ts = _inputs(seed=seed)
        got, _ = DepthLoss(lambda_ds=1.0)(res, td, tw, valid, ts)
        (g_got,) = torch.autograd.grad(got, res["depth_coarse"])
        ref = ref_cpu.depth_loss_subset(res, td, tw, valid, ts, 1.0)
        (g_ref,) = torch.autograd.grad(ref, res["depth_coarse"])
        np.testing.assert_allclose(float(got), float(ref), rtol=1e-5)
        np.testing.assert_allclose(g_got.numpy(), g_ref.numpy(), rtol=1e-5, atol=1e-9)


def test_depth_loss_empty_selections_are_zero():
    res, td, tw, valid, ts = _inputs()
    zero_valid = torch.zeros_like(valid)
    got, _ = DepthLoss()(res, td, tw, zero_valid, ts)
    assert float(got) == 0.0
    huge_std = torch.full_like(ts, 1e3)      # everything inside the expected distribution
    got, _ = DepthLoss()(res, td, tw, valid, huge_std)
    assert float(got) == 0.0
