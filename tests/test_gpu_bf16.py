"""bf16 MLP (SPNeRF(precision="bf16"), cfg.dtype = 1) vs the fp32 reference — needs an MI355X.

The bf16 path is BASELINE.json config 3's arithmetic: activations and GEMM operands in bf16
(8-bit mantissa, unit roundoff 2^-9), fp32 accumulation, fp32 heads / compositing / parameters /
gradients — the counterpart of the reference's fp16 AMP training (main.py:334-336).  fc_net.0
runs on bf16 hi/lo planes, (x_hi + x_lo)·(w_hi + w_lo) with fp32 accumulation (≈2^-17 relative
per product: the near-fp32 input precision SURVEY §8 hard part 1 asks for, at bf16 MFMA rates).
It cannot meet the 1e-4 fp32 bar by construction, so it is held to mixed-precision tolerances
against the SAME reference fixtures the fp32 path matches to 1e-4:
  * outputs: norm-relative error  ||bf16 - ref|| / ||ref|| <= OUT_TOL_KEY[key], about 3x the
    worst value measured on MI355X over CASES (tools/bf16_errors.py; the measurements are in the
    comments), so that a real regression fails;
  * gradients: norm-relative error of the whole flat gradient <= GRAD_TOL_ALL, and per parameter
    tensor of >= 64 elements <= GRAD_TOL (full-gradient fixtures; W=512 fixtures through the
    fixed random projections, error / ||grad||).  Scalar-sized gradients (σ / sun / β output
    biases: one sum over all points with heavy cancellation) are covered by the global bound only;
and it must be deterministic (fixed-order reductions, as in fp32).
"""
import numpy as np
import pytest
import torch

import golden_util as gu
import spnerf_amd
from oracle import ref_cpu
from oracle.weights import ModelDims, make_weights
from test_gpu_parity import DEV, make_model, run_case

pytestmark = pytest.mark.gpu

# per output key (suffixes _coarse / _fine / _sc dropped): the worst norm-relative error measured
# over CASES on MI355X (round 3), and the bound at ~3x it
OUT_TOL_KEY = {
    "rgb": 1.5e-3,            # 5.6e-4 (nomap_w64)
    "depth": 5e-4,            # 1.4e-4 (nomap_w64)
    "weights": 1e-3,          # 2.9e-4 (fine_sc_guided_w64)
    "transparency": 5e-4,     # 1.6e-4 (nomap_w64)
    "albedo": 1.8e-3,         # 5.7e-4 (fine_sc_guided_w64)
    "sun": 2e-3,              # 6.6e-4 (fine_w64)
    "sky": 1e-6,              # 7.6e-8: the per-ray sky MLP stays fp32
    "z_vals": 6e-4,           # 1.7e-4 (guided / fine depths follow the bf16 weights)
    "z_vals_unsort": 6e-4,    # 9.5e-5
    "beta": 2.2e-3,           # 7.2e-4 (beta_w64)
    "sem_logits": 1.5e-2,     # 4.8e-3 (fine_w64)
}
OUT_TOL = 2e-2       # the point-network check below (no per-key measurement)
GRAD_TOL = 8e-2      # per tensor; measured worst 4.6e-2 (sun_v_net.2.bias projection, c3_w512)
GRAD_TOL_ALL = 2e-2  # whole flat gradient; measured 0.4-1.6e-2 over CASES (worst fine_sc_guided_w64)
CASES = ["c1_w512", "c3_w512", "c3_w64", "beta_w64", "nomap_w64", "c3_test_w64", "c5_w512", "fine_w64",
         "fine_sc_guided_w64"]


def out_tol(key: str) -> float:
    stem = key
    for suf in ("_coarse", "_fine"):
        stem = stem[:-len(suf)] if stem.endswith(suf) else stem
    stem = stem[:-3] if stem.endswith("_sc") else stem
    return OUT_TOL_KEY[stem]


@pytest.mark.parametrize("name", CASES)
def test_bf16_render_close_to_reference(name):
    data, res, params = run_case(name, "bf16")
    keys = sorted(k[4:] for k in data if k.startswith("out_"))
    worst = {}
    for k in keys:
        got, ref = res[k].detach().cpu().numpy(), data["out_" + k]
        assert np.isfinite(got).all(), k
        if k == "z_vals_coarse" and not data["meta"]["args"]["guidedsample"]:
            # stratified depths do not depend on the network: exact (fine / guided ones do)
            gu.assert_close(f"{name}:{k}", got, ref, rtol=1e-6, atol_frac=1e-7)
        worst[k] = gu.rel_err(got, ref)
    print(name, {k: f"{v:.2e}" for k, v in worst.items()})
    bad = {k: (v, out_tol(k)) for k, v in worst.items() if v > out_tol(k)}
    assert not bad, bad


@pytest.mark.parametrize("name", CASES)
def test_bf16_gradients_close_to_reference(name):
    data, res, params = run_case(name, "bf16")
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
    total = (sq_err / sq_ref) ** 0.5
    print(name, f"flat grad rel err {total:.2e}; worst", sorted(errs.items(), key=lambda kv: -kv[1])[:4])
    assert total < GRAD_TOL_ALL, total
    bad = {k: v for k, v in errs.items() if v > GRAD_TOL}
    assert not bad, bad


@pytest.mark.parametrize("dims", [ModelDims(width=512, sem=True, beta=True), ModelDims(width=128, mapping=False)])
def test_bf16_point_network_close_to_oracle(dims):
    rng = np.random.default_rng(3)
    P = 3000
    xyz = rng.uniform(-1, 1, (P, 3)).astype(np.float32)
    sun = rng.normal(size=(P, 3)).astype(np.float32)
    lab = rng.choice([0, 1, -100] + list(range(dims.num_sem_classes)), size=P).astype(np.int64)
    t = rng.normal(size=(P, dims.t_dim)).astype(np.float32)
    m = make_model(dims, 11, "bf16")
    out = m(torch.tensor(xyz, device=DEV), input_sun_dir=torch.tensor(sun, device=DEV),
            input_t=torch.tensor(t, device=DEV) if dims.beta else None,
            input_s=torch.tensor(lab, device=DEV) if dims.sem else None).detach().cpu().numpy()
    p = ref_cpu.to_params(make_weights(dims, 11))
    ref = ref_cpu.field(p, dims, torch.tensor(xyz), torch.tensor(sun), torch.tensor(lab) if dims.sem else None,
                        torch.tensor(t) if dims.beta else None).numpy()
    cols = {"rgb": slice(0, 3), "sigma": slice(3, 4), "sun": slice(4, 5), "sky": slice(5, 8), "rest": slice(8, None)}
    errs = {k: gu.rel_err(out[:, c], ref[:, c]) for k, c in cols.items() if ref[:, c].size}
    print(errs)
    assert max(errs.values()) < OUT_TOL, errs


def test_bf16_full_size_gradients_agree_with_fp32():
    """Config-3 shape (1024 rays, 64+64 guided, sc, sem, W=512): bf16 vs fp32 HIP path on the
    same draws — outputs and every parameter gradient (the fp32 path is the parity-pinned one)."""
    from test_gpu_parity import gu_rays
    dims = ModelDims(width=512, sem=True)
    args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                    sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    B = 1024
    rays = torch.tensor(gu_rays(B, 9), device=DEV)
    g = torch.Generator(device="cpu").manual_seed(0)
    valid = (torch.rand(B, generator=g) < 0.68).long().to(DEV)
    td = torch.stack([rays[:, 7] * 0.5, torch.ones(B, device=DEV)], 1)
    tstd = torch.full((B,), 0.01, device=DEV)
    sem = torch.randint(0, 3, (B,), generator=g).to(DEV)
    outs = {}
    for prec in ("fp32", "bf16"):
        model = make_model(dims, 2, prec)
        torch.manual_seed(123)  # the default device random source draws the same u's for both runs
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sem, mode="train",
                                     valid_depth=valid, target_depths=td, target_std=tstd)
        loss = ((res["rgb_coarse"] - 0.5) ** 2).mean() + res["sun_sc_coarse"].mean() + res["sem_logits_coarse"].square().mean()
        loss.backward()
        outs[prec] = ({k: v.detach().cpu() for k, v in res.items()}, {n: p.grad.cpu() for n, p in model.named_parameters()})
    (r32, g32), (r16, g16) = outs["fp32"], outs["bf16"]
    for k in ("rgb_coarse", "depth_coarse", "sem_logits_coarse", "sun_sc_coarse"):
        e = gu.rel_err(r16[k].numpy(), r32[k].numpy())
        print(k, f"{e:.2e}")
        assert e < out_tol(k), (k, e)
    errs = {n: gu.rel_err(g16[n].numpy(), g32[n].numpy()) for n in g32 if g32[n].abs().sum() > 0}
    print("worst grads", sorted(errs.items(), key=lambda kv: -kv[1])[:6])
    assert max(errs.values()) < GRAD_TOL, errs


def test_bf16_deterministic():
    outs = []
    for _ in range(2):
        data, res, params = run_case("c3_w512", "bf16")
        loss = sum(v.sum() for k, v in res.items() if v.requires_grad)
        loss.backward()
        outs.append([res[k].detach().cpu() for k in sorted(res)] + [params[n].grad.cpu() for n in sorted(params)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["c3_w512", "c5_w512"])
def test_zsave_option_close_to_default(name):
    """Option zsave (off by default): the training forward saves only the fp16
    pre-activation Z of trunk layers 1..L-2, the backward recomputes sin(Z) / cos(Z).  Same
    arithmetic up to where Z is rounded: outputs within 2e-3 and the flat gradient within the
    spread that benign rounding changes give on these fixtures (l0_split=0 moves c1_w512's
    gradient error 1.5e-2 -> 2.1e-2), and still within GRAD_TOL_ALL of the reference."""
    from spnerf_amd import _lib
    runs = {}
    try:
        for z in (0, 1):
            _lib.set_option("zsave", z)
            data, res, params = run_case(name, "bf16")
            shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
            R = gu.projection_weights(shapes)
            loss = sum((res[k] * torch.tensor(R[k], device=DEV)).sum() for k in sorted(R))
            loss.backward()
            runs[z] = ({k: v.detach().cpu().numpy() for k, v in res.items()},
                       np.concatenate([p.grad.detach().double().cpu().numpy().ravel() for n, p in sorted(params.items())]))
    finally:
        _lib.set_option("zsave", 0)
    (o0, g0), (o1, g1) = runs[0], runs[1]
    worst = max(gu.rel_err(o1[k], o0[k]) for k in o0 if o0[k].size and np.any(o0[k]))
    gd = float(np.linalg.norm(g1 - g0) / np.linalg.norm(g0))
    print(name, f"outputs {worst:.2e} flat grad {gd:.2e}")
    assert worst < 2e-3
    assert gd < GRAD_TOL_ALL
