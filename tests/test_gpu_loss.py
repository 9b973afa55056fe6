"""The fused training loss (csrc/loss.hip, spnerf_amd.losses.FusedRenderLoss) against the
losses module pinned to the reference's metrics.py (tests/test_losses.py): value, every term and
every upstream gradient, on render-shaped inputs (sun_sc a strided view of the MLP output, as in
a render) and on a real render; data-parallel shards average to the global loss (needs an MI355X)."""
import numpy as np
import pytest
import torch

import golden_util as gu
from spnerf_amd import losses as L

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def inputs(B=300, S=128, C=3, seed=0, NO=11):
    g = torch.Generator().manual_seed(seed)
    out = torch.rand(B * S, NO, generator=g)
    w = torch.rand(B, S, generator=g) ** 3
    w = w / w.sum(1, keepdim=True) * (0.6 + 0.4 * torch.rand(B, 1, generator=g))
    z = torch.sort(torch.rand(B, S, generator=g) * 0.2, 1)[0]
    res = {"rgb_coarse": torch.rand(B, 3, generator=g), "depth_coarse": (w * z).sum(1), "weights_coarse": w,
           "z_vals_coarse": z, "transparency_sc_coarse": torch.cumprod(0.8 + 0.2 * torch.rand(B, S, generator=g), 1),
           "weights_sc_coarse": 0.1 * torch.rand(B, S, generator=g), "sem_logits_coarse": torch.randn(B, C, generator=g)}
    tgt = torch.rand(B, 3, generator=g)
    td = torch.stack([res["depth_coarse"] * (0.7 + 0.6 * torch.rand(B, generator=g)), 0.2 + 0.8 * torch.rand(B, generator=g)], 1)
    valid = (torch.rand(B, generator=g) < 0.7).long()
    tstd = 1e-3 + 0.02 * torch.rand(B, generator=g)
    labels = torch.tensor(np.random.default_rng(seed).choice([0, 1, 2, -100], size=B, p=[0.3, 0.3, 0.25, 0.15]))
    d = lambda t: t.to(DEV)
    out = d(out).requires_grad_(True)
    r = {k: d(v).requires_grad_(k in ("rgb_coarse", "depth_coarse", "sem_logits_coarse")) for k, v in res.items()}
    r["sun_sc_coarse"] = out.view(B, S, NO)[..., 4:5]
    return r, out, d(tgt), d(td), d(valid), d(tstd), d(labels)


def reference(r, tgt, td, valid, tstd, labels, lsc, lds, lss):
    loss, t1 = L.SNerfLoss(lambda_sc=lsc)(r, tgt)
    ld, t2 = L.DepthLoss(lds, usealldepth=False)(r, td[:, 0], td[:, 1], valid, tstd)
    ls, t3 = L.SemanticLoss(lss)(r, labels)
    return loss + ld + ls, {**t1, **t2, **t3}


@pytest.mark.parametrize("lsc,lds,lss", [(0.1, 1.0, 1.0), (0.05, 0.0, 0.04), (0.0, 0.7, 0.0)])
def test_fused_loss_matches_reference_losses(lsc, lds, lss):
    vals = {}
    for impl in ("ref", "fused"):
        r, out, tgt, td, valid, tstd, labels = inputs()
        if impl == "ref":
            loss, terms = reference(r, tgt, td, valid, tstd, labels, lsc, lds, lss)
        else:
            loss, terms = L.FusedRenderLoss(lsc, lds, lss)(r, tgt, td, valid, tstd, labels)
        (2.5 * loss).backward()
        vals[impl] = (float(loss), {k: float(v) for k, v in terms.items()},
                      {k: (r[k].grad if r[k].grad is not None else torch.zeros_like(r[k])).cpu().numpy()
                       for k in ("rgb_coarse", "depth_coarse", "sem_logits_coarse")},
                      out.grad.cpu().numpy() if out.grad is not None else None)
    (lr, tr, gr, orr), (lf, tf, gf, of) = vals["ref"], vals["fused"]
    np.testing.assert_allclose(lf, lr, rtol=1e-5)
    for k, v in tr.items():
        np.testing.assert_allclose(tf[k], v, rtol=1e-5, atol=1e-7, err_msg=k)
    for k, v in gr.items():
        gu.assert_close(k, gf[k], v, rtol=1e-5, atol_frac=1e-6)
    if lsc > 0:
        gu.assert_close("sun_sc (through the out view)", of, orr, rtol=1e-5, atol_frac=1e-6)


def test_fused_loss_shards_average_to_the_global_loss():
    r, out, tgt, td, valid, tstd, labels = inputs(B=256)
    glob, _ = L.FusedRenderLoss(0.1, 1.0, 1.0)(r, tgt, td, valid, tstd, labels)
    parts = []
    for k in range(2):
        sl = slice(128 * k, 128 * k + 128)
        rk = {n: v[sl] for n, v in r.items()}
        parts.append(L.FusedRenderLoss(0.1, 1.0, 1.0)(rk, tgt[sl], td[sl], valid[sl], tstd[sl], labels[sl],
                                                      labels_global=labels, world=2)[0])
    np.testing.assert_allclose(float(sum(parts) / 2), float(glob), rtol=1e-5)


def test_fused_loss_deterministic():
    r, out, tgt, td, valid, tstd, labels = inputs(B=1000)
    a = L.FusedRenderLoss(0.1, 1.0, 1.0)(r, tgt, td, valid, tstd, labels)[0]
    b = L.FusedRenderLoss(0.1, 1.0, 1.0)(r, tgt, td, valid, tstd, labels)[0]
    assert torch.equal(a, b)


def test_fused_loss_label_errors_are_nan_not_silent():
    """Labels outside [0, C) other than -100 (torch raises there) make the loss and those rays'
    logit gradients NaN; a batch with no valid label gives a NaN CE term (torch's mean over
    nothing) and zero logit gradients; target_valid_depth=None means every ray has a prior."""
    r, out, tgt, td, valid, tstd, labels = inputs(B=64, S=32)
    bad = labels.clone()
    bad[5] = 3
    loss, terms = L.FusedRenderLoss(0.1, 1.0, 1.0)(r, tgt, td, valid, tstd, bad)
    loss.backward()
    assert torch.isnan(loss) and torch.isnan(terms["coarse_ss"])
    g = r["sem_logits_coarse"].grad
    assert torch.isnan(g[5]).all() and torch.isfinite(torch.cat([g[:5], g[6:]])).all()
    r, out, tgt, td, valid, tstd, labels = inputs(B=64, S=32)
    loss, terms = L.FusedRenderLoss(0.1, 1.0, 1.0)(r, tgt, td, valid, tstd, torch.full_like(labels, -100))
    loss.backward()
    ref = L.SemanticLoss(1.0)(r, torch.full_like(labels, -100))[0]
    assert torch.isnan(terms["coarse_ss"]) and torch.isnan(ref)
    assert float(r["sem_logits_coarse"].grad.abs().sum()) == 0.0
    r, out, tgt, td, valid, tstd, labels = inputs(B=64, S=32)
    a = L.FusedRenderLoss(0.0, 1.0, 0.0)(r, tgt, td, None, tstd)[0]
    b = L.FusedRenderLoss(0.0, 1.0, 0.0)(r, tgt, td, torch.ones_like(valid), tstd)[0]
    assert float(a) == float(b)
