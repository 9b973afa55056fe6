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
