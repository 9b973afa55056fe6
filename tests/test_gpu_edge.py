"""Edge batches through the whole render path on the HIP kernels — needs an MI355X.

An empty batch (0 rays: every launch of the step sees zero rays or points) must return outputs of
the reference's shapes with 0 rows and a backward that leaves every parameter gradient zero; a
single ray must render as it does inside a larger batch (rays are independent: the same ray in a
batch of 97 renders bit for bit equal in fp32).  Train mode (guided sampling on / off, solar pass
on, semantic head on) and evaluation without gradients, fp32 and bf16."""
import pytest
import torch

import golden_util as gu
import spnerf_amd
from oracle.weights import ModelDims
from test_gpu_parity import DEV, gu_rays, make_model

pytestmark = pytest.mark.gpu


def _args(guided, n_samples=64):
    return gu.args_of({"args": dict(n_samples=n_samples, n_importance=0, model="sp-nerf", beta=False,
                                    guidedsample=guided, sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120,
                                    noise_std=0.0)})


def _inputs(rays, guided):
    n = rays.shape[0]
    g = torch.Generator(device="cpu").manual_seed(8)
    kw = {}
    if guided:
        kw = dict(valid_depth=(torch.rand(n, generator=g) < 0.7).long().to(DEV),
                  target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n, device=DEV)], 1),
                  target_std=torch.full((n,), 0.01, device=DEV))
    labels = torch.randint(0, 3, (n,), generator=g).to(DEV)
    return labels, kw


def _rays(n):
    base = torch.tensor(gu_rays(max(n, 1), 31), device=DEV)
    return base[:n].contiguous()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("guided", [True, False])
def test_empty_batch_train_step(precision, guided):
    model = make_model(ModelDims(width=512, sem=True), 9, precision)
    rays = _rays(0)
    labels, kw = _inputs(rays, guided)
    res = spnerf_amd.render_rays({"coarse": model}, _args(guided), rays, None, semantics=labels, mode="train", **kw)
    assert "rgb_coarse" in res and "sun_sc_coarse" in res
    for k, v in res.items():
        assert v.shape[0] == 0, (k, tuple(v.shape))
    loss = sum(v.float().sum() for k, v in sorted(res.items()) if v.requires_grad)
    loss.backward()
    torch.cuda.synchronize()
    assert float(loss.detach()) == 0.0
    for n, p in model.named_parameters():
        assert p.grad is None or not p.grad.any(), n


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_empty_batch_eval(precision):
    model = make_model(ModelDims(width=512, sem=True), 9, precision)
    rays = _rays(0)
    labels, _ = _inputs(rays, False)
    with torch.no_grad():
        res = spnerf_amd.render_rays({"coarse": model}, _args(True), rays, None, semantics=labels, mode="test")
    torch.cuda.synchronize()
    assert res and all(v.shape[0] == 0 for v in res.values())


@pytest.mark.parametrize("guided,ray", [(False, 5), (True, 0)])
def test_single_ray_equals_its_row_in_a_batch(guided, ray):
    """fp32: one ray of a 97-ray batch rendered alone gives the same outputs bit for bit.  The
    Philox draws are keyed by the global ray id (``ray_offset``), so both renders draw the same
    depths.  Guided sampling clamps every ray's window to the FIRST ray's bounds (the reference's
    ``rendering.py:95,113`` — near[0, 0], far[0, 0]), so there the lone ray is ray 0."""
    model = make_model(ModelDims(width=512, sem=True), 9, "fp32")
    rays = _rays(97)
    labels, kw = _inputs(rays, guided)
    outs = []
    for idx, off in ((torch.arange(97, device=DEV), 0), (torch.tensor([ray], device=DEV), ray)):
        sub = {k: v[idx] for k, v in kw.items()}
        with torch.no_grad(), spnerf_amd.random_source(spnerf_amd.PhiloxRandom(seed=5, ray_offset=off)):
            outs.append(spnerf_amd.render_rays({"coarse": model}, _args(guided), rays[idx].contiguous(), None,
                                               semantics=labels[idx], mode="train", **sub))
    full, one = outs
    assert sorted(full) == sorted(one)
    for k in one:
        assert torch.equal(full[k][ray:ray + 1], one[k]), k
