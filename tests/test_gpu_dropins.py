"""The public drop-ins outside render_rays, on the HIP path, against the reference's own outputs
(fixture dropins_w64, tests/golden/gen_golden.py::dropins) — needs an MI355X:

* ``inference(model, args, rays_xyz, z_vals, ...)`` on explicit sample positions
  (models/spnerf.py:63-159) with σ noise and semantics: outputs and full gradients;
* ``compute_samples_around_depth`` (modules/rendering.py:76-89) and ``GenerateGuidedSamples``
  (:92-116) in test and train mode — samples in the reference's DRAW order;
* ``load_model(args)`` (models/__init__.py:4-16) building the module that renders a fixture;
* autograd semantics of the packed weights: a backward uses the weights of its own forward
  even when the parameters change and another forward re-packs in between.
"""
import types

import numpy as np
import pytest
import torch

import golden_util as gu
import spnerf_amd
from spnerf_amd import ReplayRandom, random_source
from oracle.weights import ModelDims, make_weights
from test_gpu_parity import DEV, make_model, run_case

pytestmark = pytest.mark.gpu


def fixture():
    with np.load(f"{gu.GOLDEN}/dropins_w64.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_inference_dropin_matches_reference():
    d = fixture()
    model = make_model(ModelDims(width=64, sem=True), 12)
    rays = torch.tensor(d["rays"], device=DEV)
    args = types.SimpleNamespace(n_samples=32, chunk=5120, noise_std=float(d["noise_std"]))
    with random_source(ReplayRandom([("randn", d["rng00_randn"])])) as src:
        res = spnerf_amd.inference(model, args, torch.tensor(d["xyz"], device=DEV), torch.tensor(d["z"], device=DEV),
                                   sun_d=rays[:, 8:11], semantics=torch.tensor(d["in_semantics"], device=DEV))
    assert src.used == 1
    keys = sorted(k[4:] for k in d if k.startswith("out_"))
    assert sorted(res) == keys
    for k in keys:
        gu.assert_close(k, res[k].detach().cpu().numpy(), d["out_" + k], rtol=1e-4, atol_frac=1e-5)
    R = gu.projection_weights({k: tuple(v.shape) for k, v in res.items() if v.requires_grad})
    sum((res[k] * torch.tensor(R[k], device=DEV)).sum() for k in sorted(R)).backward()
    for n, p in model.named_parameters():
        gu.assert_close("grad " + n, p.grad.cpu().numpy(), d["grad_" + n], rtol=1e-4, atol_frac=1e-4)


def test_guided_sampling_dropins_match_reference_in_draw_order():
    d = fixture()
    rays = torch.tensor(d["rays"], device=DEV)
    z = torch.tensor(d["z"], device=DEV)
    S = z.shape[1]
    rd = {"depth": torch.tensor(d["out_depth"], device=DEV), "weights": torch.tensor(d["out_weights"], device=DEV)}
    near, far = rays[:, 6:7], rays[:, 7:8]
    with random_source(ReplayRandom([("rand", d["csad_u"])])):
        zc = spnerf_amd.compute_samples_around_depth(rd, S, z, 1.0, near[0, 0], far[0, 0])
    gu.assert_close("compute_samples_around_depth", zc.cpu().numpy(), d["csad_out"], rtol=1e-5, atol_frac=1e-6)
    with random_source(ReplayRandom([("rand", d["ggs_test_u"])])):
        zt = spnerf_amd.GenerateGuidedSamples(rd, z, S, 1.0, near, far, mode="test")
    gu.assert_close("GenerateGuidedSamples test", zt.cpu().numpy(), d["ggs_test_out"], rtol=1e-5, atol_frac=1e-6)
    with random_source(ReplayRandom([("rand", d["ggs_train_u0"]), ("rand", d["ggs_train_u1"])])) as src:
        ztr = spnerf_amd.GenerateGuidedSamples(rd, z, S, 1.0, near, far, mode="train",
                                               valid_depth=torch.tensor(d["in_valid_depth"], device=DEV),
                                               target_depths=torch.tensor(d["in_target_depths"], device=DEV),
                                               target_std=torch.tensor(d["in_target_std"], device=DEV))
    assert src.used == 2
    gu.assert_close("GenerateGuidedSamples train", ztr.cpu().numpy(), d["ggs_train_out"], rtol=1e-5, atol_frac=1e-6)
    assert not bool((ztr.cpu().diff(dim=-1) >= 0).all()), "draw order, not sorted"
    with pytest.raises(AssertionError):
        spnerf_amd.GenerateGuidedSamples(rd, z, S, 1.0, near, far, mode="train")


def test_load_model_renders_a_fixture():
    """The factory builds a module the render path accepts; with the fixture's weights loaded
    it renders the C3-flags fixture like SPNeRF(...) does."""
    data = gu.load("c3_w64")
    dims = gu.dims_of(data["meta"])
    args = types.SimpleNamespace(model="sp-nerf", num_sem_classes=dims.num_sem_classes,
                                 s_embedding_factor=dims.s_embedding_factor, fc_layers=dims.layers, fc_units=dims.width,
                                 mapping=dims.mapping, t_embbeding_tau=dims.t_dim, beta=dims.beta, sem=dims.sem)
    m = spnerf_amd.load_model(args)
    m.load_state_dict({k: torch.tensor(v) for k, v in make_weights(dims, data["meta"]["seed"]).items()})
    m = m.to(DEV)
    rargs = gu.args_of(data["meta"])
    kw = dict(valid_depth=torch.tensor(data["in_valid_depth"], device=DEV),
              target_depths=torch.tensor(data["in_target_depths"], device=DEV),
              target_std=torch.tensor(data["in_target_std"], device=DEV))
    with random_source(ReplayRandom(gu.draws_of(data))):
        res = spnerf_amd.render_rays({"coarse": m}, rargs, torch.tensor(data["rays"], device=DEV), None,
                                     semantics=torch.tensor(data["in_semantics"], device=DEV), mode="train", **kw)
    for k in ("rgb_coarse", "depth_coarse", "sem_logits_coarse", "sun_sc_coarse"):
        gu.assert_close(k, res[k].detach().cpu().numpy(), data["out_" + k], rtol=1e-4, atol_frac=1e-5)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_backward_uses_the_weights_of_its_forward(precision):
    """forward(A) → parameters changed in place (no version bump, like a fused optimizer) →
    forward(B) re-packs → backward of the first graph: its gradients equal a clean
    forward/backward at A (each saving forward packs into a buffer of its own)."""
    data = gu.load("c1_w64")
    meta = data["meta"]
    dims, args = gu.dims_of(meta), gu.args_of(meta)
    rays = torch.tensor(data["rays"], device=DEV)

    def fwd(m):
        with random_source(ReplayRandom(gu.draws_of(data))):
            return spnerf_amd.render_rays({"coarse": m}, args, rays, None, mode=meta["mode"])

    clean = make_model(dims, meta["seed"], precision)
    fwd(clean)["rgb_coarse"].sum().backward()
    model = make_model(dims, meta["seed"], precision)
    res_a = fwd(model)
    with torch.no_grad():
        for p in model.parameters():
            p.data.mul_(1.5)             # in place, behind autograd's back
    res_b = fwd(model)
    res_a["rgb_coarse"].sum().backward()
    for (n, p), q in zip(model.named_parameters(), clean.parameters()):
        assert torch.equal(p.grad, q.grad), n
    assert not torch.equal(res_a["rgb_coarse"], res_b["rgb_coarse"])
