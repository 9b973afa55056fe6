"""The direct (flat-buffer) gradient path of the MLP backward is opt-in (SPNeRF.use_flat_grads):
off by default the gradients return through autograd, so torch.autograd.grad works and frozen
parameters never receive a .grad; on, the backward adds into one flat buffer whose views are the
.grads, with the same values — and it stays off for a model with a frozen parameter."""
import pytest
import torch

import golden_util as gu
import spnerf_amd
from oracle.weights import ModelDims
from test_gpu_parity import DEV, gu_rays, make_model

pytestmark = pytest.mark.gpu


def _loss(model, n_rays=64):
    args = gu.args_of({"args": dict(n_samples=32, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    rays = torch.tensor(gu_rays(n_rays, 4), device=DEV)
    torch.manual_seed(7)
    res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, mode="train")
    return (res["rgb_coarse"] ** 2).mean() + res["sun_sc_coarse"].mean()


def test_flat_grads_opt_in_matches_autograd():
    dims = ModelDims(width=64)
    m = make_model(dims, 3)
    assert not m.flat_grads
    params = list(m.parameters())
    ref = torch.autograd.grad(_loss(m), params, allow_unused=True)
    assert all(p.grad is None for p in params)          # autograd.grad leaves .grad alone
    m.use_flat_grads()
    _loss(m).backward()
    base = params[0].grad._base
    assert base is not None and all(p.grad._base is base for p in params)
    for p, r in zip(params, ref):
        torch.testing.assert_close(p.grad, torch.zeros_like(p) if r is None else r, rtol=1e-5, atol=1e-6)


def test_flat_grads_never_touch_frozen_parameters():
    m = make_model(ModelDims(width=64), 3).use_flat_grads()
    frozen = m.sigma_from_xyz[0].weight
    frozen.requires_grad_(False)
    _loss(m).backward()
    assert frozen.grad is None
    assert all(p.grad is not None for n, p in m.named_parameters() if p.requires_grad and "semantic" not in n)


@pytest.mark.parametrize("sem", [False, True])
def test_deferred_trunk_weight_gradients_match_per_pass(sem):
    """bf16 MLP, main + solar pass: with flat gradients the two backwards leave the trunk's weight
    gradients to one two-segment GEMM per layer (spnerf_mlp_trunk_wgrad, run by an autograd
    callback).  Same gradient as one GEMM per pass up to fp32 summation order."""
    import types
    args = types.SimpleNamespace(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    rays = torch.tensor(gu_rays(96, 4), device=DEV)
    g = torch.Generator().manual_seed(3)
    depths = torch.rand(96, 2, generator=g).to(DEV) * 0.5 + 0.2
    valid = (torch.rand(96, generator=g) > 0.3).long().to(DEV)
    sems = torch.randint(0, 3, (96,), generator=g).to(DEV)
    grads = {}
    for defer in (False, True):
        torch.manual_seed(0)
        m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=sem,
                              precision="bf16").to(DEV).use_flat_grads()
        m.defer_trunk_wgrad = defer
        with spnerf_amd.random_source(spnerf_amd.PhiloxRandom(seed=5)):
            res = spnerf_amd.render_rays({"coarse": m}, args, rays, None, semantics=sems if sem else None, mode="train",
                                         valid_depth=valid, target_depths=depths, target_std=depths[:, 1] * 0 + 0.01)
        loss = (res["rgb_coarse"] ** 2).mean() + res["sun_sc_coarse"].mean() + res["depth_coarse"].mean()
        loss.backward()
        grads[defer] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    num = den = 0.0
    for n, a in grads[False].items():
        b = grads[True][n]
        num += float(((a - b).double() ** 2).sum())
        den += float((a.double() ** 2).sum())
        if a.numel() >= 64 and float(a.norm()) > 0:
            assert float((a - b).norm() / a.norm()) <= 1e-3, n
    assert (num / den) ** 0.5 <= 1e-5
    assert float(grads[True]["fc_net.2.weight"].norm()) > 0


def _deferred_grads(tn_group, n_rays=96, rounds=1, beta=False, defer_heads=1):
    """Flat bf16 gradients of a main + solar render with the deferred trunk weight gradients, and
    the number of DMA weight-gradient launches they took."""
    import types
    from spnerf_amd import _lib
    args = types.SimpleNamespace(n_samples=64, n_importance=0, model="sp-nerf", beta=beta, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    rays = torch.tensor(gu_rays(n_rays, 4), device=DEV)
    g = torch.Generator().manual_seed(3)
    depths = torch.rand(n_rays, 2, generator=g).to(DEV) * 0.5 + 0.2
    valid = (torch.rand(n_rays, generator=g) > 0.3).long().to(DEV)
    sems = torch.randint(0, 3, (n_rays,), generator=g).to(DEV)
    ts = torch.randint(0, 4, (n_rays,), generator=g).to(DEV)
    # (tn_group_rounds is an ablation-build switch; the product library runs its automatic choice,
    # rounds = 0, which is 1 block per CU below 2^16 points per split — so rounds 0 and, at these
    # small sizes, 1 need no switch; 2 skips in the product build)
    opts = {"tn_group": tn_group, "defer_heads": defer_heads}
    if _lib.has_option("tn_group_rounds") or rounds not in (0, 1):
        opts["tn_group_rounds"] = rounds
    names = tuple(opts)
    old = [_lib.get_option(k) for k in names]
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        torch.manual_seed(0)
        m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True, beta=beta,
                              t_embedding_dims=4 if beta else 16, precision="bf16").to(DEV).use_flat_grads()
        m.defer_trunk_wgrad = True
        models = {"coarse": m}
        if beta:
            torch.manual_seed(1)
            models["t"] = torch.nn.Embedding(4, 4).to(DEV)
        with spnerf_amd.random_source(spnerf_amd.PhiloxRandom(seed=5)):
            res = spnerf_amd.render_rays(models, args, rays, ts if beta else None, semantics=sems, mode="train",
                                         valid_depth=valid, target_depths=depths, target_std=depths[:, 1] * 0 + 0.01)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        torch.cuda.synchronize()
        _lib.prof_reset()
        _lib.prof_enable(True)
        loss.backward()
        torch.cuda.synchronize()
        _lib.prof_enable(False)
        launches = _lib.prof_read("gemm_tn_bf16d")["launches"] if "gemm_tn_bf16d" in _lib.prof_classes() else 0
        return {n: p.grad.detach().clone() for n, p in m.named_parameters()}, launches
    finally:
        for k, v in zip(names, old):
            _lib.set_option(k, v)


@pytest.mark.parametrize("group,rounds,beta,n_rays", [(4, 1, False, 96), (9, 1, False, 96), (9, 2, False, 96), (10, 1, True, 96),
                                                    (6, 2, True, 96), (9, 0, False, 2048)])
def test_grouped_trunk_weight_gradients_match(group, rounds, beta, n_rays):
    """Option tn_group: the deferred output-head (G / Q, defer_heads), sun_v and trunk-layer
    weight-gradient GEMMs (the skip layer's H part; its PE tail on the narrow kernel) run `group`
    per launch of the DMA kernel, splits in proportion to their points (`rounds` blocks per CU).  Fewer launches, the same gradients up to fp32
    summation order."""
    # (2 048 rays: 2^18 points per pass, the bench's sizes — the ungrouped skip layer takes the
    # split-tail path, the grouped one the paired narrow launch, 2 blocks per CU with rounds 0)
    g0, _ = _deferred_grads(1, n_rays, beta=beta, defer_heads=0)   # the heads' weight gradients per pass
    g1, n1 = _deferred_grads(1, n_rays, beta=beta)
    g2, n2 = _deferred_grads(group, n_rays, rounds=rounds, beta=beta)
    for n, a in g0.items():   # deferred heads (per segment, ungrouped) = per pass up to summation order
        if a.numel() >= 64 and float(a.norm()) > 0:
            assert float((a - g1[n]).norm() / a.norm()) <= 1e-4, n
    assert n2 < n1, (n1, n2)
    num = den = 0.0
    for n, a in g1.items():
        b = g2[n]
        assert torch.isfinite(b).all(), n
        num += float(((a - b).double() ** 2).sum())
        den += float((a.double() ** 2).sum())
        if a.numel() >= 64 and float(a.norm()) > 0:
            assert float((a - b).norm() / a.norm()) <= 1e-4, n
    assert (num / den) ** 0.5 <= 1e-5
    # deterministic: the same grouping twice is bit for bit the same
    g3, _ = _deferred_grads(group, n_rays, rounds=rounds, beta=beta)
    for n in g2:
        assert torch.equal(g2[n], g3[n]), n
