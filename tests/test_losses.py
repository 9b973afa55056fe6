"""spnerf_amd.losses (the drop-in for modules/metrics.py) against the reference's own values and
gradients (tests/golden/losses.npz, generated from metrics.py by gen_golden.py::losses), on the
CPU: SNerfLoss (+ solar terms, + fine), SatNerfLoss (β), DepthLoss (subset MSE, subset GNLL,
use-all-depth, + fine), SemanticLoss (ignore_index, + fine), psnr."""
import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import ref_cpu
from spnerf_amd import losses as L


def fixture():
    with np.load(f"{gu.GOLDEN}/losses.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


D = fixture()
CO = [k[3:] for k in D if k.startswith("in_") and k.endswith("_coarse")]
ALL = [k[3:] for k in D if k.startswith("in_") and (k.endswith("_coarse") or k.endswith("_fine"))]
T = lambda k: torch.tensor(D["in_" + k])
CASES = {
    "snerf_sc": (CO, lambda x: L.SNerfLoss(lambda_sc=0.1)(x, T("targets"))),
    "snerf_fine": (ALL, lambda x: L.SNerfLoss(lambda_sc=0.05)(x, T("targets"))),
    "satnerf_sc": (CO, lambda x: L.SatNerfLoss(lambda_sc=0.1)(x, T("targets"))),
    "satnerf_fine": (ALL, lambda x: L.SatNerfLoss(lambda_sc=0.0)(x, T("targets"))),
    "depth_subset": (CO, lambda x: L.DepthLoss(1.0, usealldepth=False)(x, T("depth_t"), T("depth_w"), T("valid"), T("dstd"))),
    "depth_subset_fine": (ALL, lambda x: L.DepthLoss(0.7, usealldepth=False)(x, T("depth_t"), T("depth_w"), T("valid"),
                                                                          T("dstd"))),
    "depth_gnll": (CO, lambda x: L.DepthLoss(1.0, GNLL=True, usealldepth=False)(x, T("depth_t"), T("depth_w"), T("valid"),
                                                                                T("dstd"))),
    "depth_all": (ALL, lambda x: L.DepthLoss(1.0, usealldepth=True)(x, T("depth_t"), T("depth_w"), T("valid"), T("dstd"))),
    "sem": (CO, lambda x: L.SemanticLoss(lambda_ss=0.04)(x, T("labels"))),
    "sem_fine": (ALL, lambda x: L.SemanticLoss(lambda_ss=1.0)(x, T("labels"))),
}


@pytest.mark.parametrize("tag", sorted(CASES))
def test_loss_values_and_gradients_match_reference(tag):
    keys, fn = CASES[tag]
    x = {k: torch.tensor(D["in_" + k], requires_grad=True) for k in keys}
    loss, ld = fn(x)
    loss.backward()
    np.testing.assert_allclose(float(loss), float(D[f"{tag}|loss"]), rtol=1e-5, atol=1e-8)
    terms = {k.split("|")[2] for k in D if k.startswith(f"{tag}|term|")}
    assert set(ld) == terms, (sorted(ld), sorted(terms))
    for k in terms:
        np.testing.assert_allclose(float(ld[k]), float(D[f"{tag}|term|{k}"]), rtol=1e-5, atol=1e-8, err_msg=k)
    for k, v in x.items():
        g = v.grad.numpy() if v.grad is not None else np.zeros_like(D["in_" + k])
        gu.assert_close(f"{tag} grad {k}", g, D[f"{tag}|grad|{k}"], rtol=1e-4, atol_frac=1e-6)


def test_psnr_matches_reference():
    np.testing.assert_allclose(float(L.psnr(T("rgb_coarse"), T("targets"))), float(D["psnr"]), rtol=1e-6)


def test_load_loss():
    import types
    assert isinstance(L.load_loss(types.SimpleNamespace(model="sp-nerf", beta=True, sc_lambda=0.1)), L.SatNerfLoss)
    assert isinstance(L.load_loss(types.SimpleNamespace(model="sp-nerf", beta=False, sc_lambda=0.1)), L.SNerfLoss)
    with pytest.raises(ValueError):
        L.load_loss(types.SimpleNamespace(model="nerf", beta=False, sc_lambda=0.0))


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


def test_depth_loss_subset_matches_the_oracle():
    for seed in range(4):
        res, td, tw, valid, ts = _inputs(seed=seed)
        got, _ = L.DepthLoss(lambda_ds=1.0, usealldepth=False)(res, td, tw, valid, ts)
        (g_got,) = torch.autograd.grad(got, res["depth_coarse"])
        ref = ref_cpu.depth_loss_subset(res, td, tw, valid, ts, 1.0)
        (g_ref,) = torch.autograd.grad(ref, res["depth_coarse"])
        np.testing.assert_allclose(float(got), float(ref), rtol=1e-5)
        np.testing.assert_allclose(g_got.numpy(), g_ref.numpy(), rtol=1e-5, atol=1e-9)


def test_depth_loss_empty_selections_are_zero():
    res, td, tw, valid, ts = _inputs()
    got, _ = L.DepthLoss(usealldepth=False)(res, td, tw, torch.zeros_like(valid), ts)
    assert float(got) == 0.0
    got, _ = L.DepthLoss(usealldepth=False)(res, td, tw, valid, torch.full_like(ts, 1e3))  # all inside
    assert float(got) == 0.0


def test_gnll_ray_left_out_with_zero_spread_keeps_gradient_finite():
    """A ray with one-hot weights (zero predicted spread) that the subset rule leaves out — no
    depth prior — puts no NaN into the GNLL gradient (the reference computes σ_pred only on the
    applied rays, metrics.py:90-102)."""
    S = 8
    w = torch.zeros(2, S)
    w[0, 3] = 1.0                      # zero spread, invalid prior → left out
    w[1] = torch.full((S,), 1.0 / S)   # spread out, applied
    w.requires_grad_(True)
    z = torch.linspace(0.1, 0.9, S).repeat(2, 1)
    depth = (w * z).sum(1)
    res = {"weights_coarse": w, "z_vals_coarse": z, "depth_coarse": depth}
    loss, _ = L.DepthLoss(1.0, GNLL=True, usealldepth=False)(res, torch.tensor([0.5, 0.2]), torch.ones(2),
                                                             torch.tensor([0, 1]), torch.tensor([0.01, 0.01]))
    loss.backward()
    assert torch.isfinite(loss) and torch.isfinite(w.grad).all()
    assert float(w.grad[0].abs().sum()) == 0.0


def test_oracle_train_loss_is_the_reference_sum():
    """oracle/ref_cpu.train_loss (the CPU baseline's loss: main.py:143-174) = the reference's
    SNerfLoss(0.1) + DepthLoss(1.0, subset) + SemanticLoss(0.04) values on the same inputs."""
    x = {k: torch.tensor(D["in_" + k]) for k in CO}
    depths = torch.stack([T("depth_t"), T("depth_w")], 1)
    got = ref_cpu.train_loss(x, T("targets"), depths, T("valid"), T("dstd"), T("labels"), 0.1, 1.0, 0.04)
    want = float(D["snerf_sc|loss"]) + float(D["depth_subset|loss"]) + float(D["sem|loss"])
    np.testing.assert_allclose(float(got), want, rtol=1e-5, atol=1e-8)
