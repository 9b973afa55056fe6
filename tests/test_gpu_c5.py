"""Config 5 (BASELINE.json configs[4]): whole-image inference — 128 stratified samples per ray,
semantic head on (C=3), W=512, bf16 MLP, no grad — on the HIP path (needs an MI355X).

* against the reference: fixture c5_w512 (64 rays of the C5 flags rendered by the reference's
  own render_rays, tests/golden/gen_golden.py) through render_rays(mode="test") under
  torch.no_grad(), i.e. the fused inference trunk; fp32 at the 1e-4 bar, bf16 at the
  mixed-precision bound of test_gpu_bf16 (OUT_TOL, norm-relative);
* at full chunk size (32 768 rays x 128 samples = 4.2 M points, the bench's per-step chunk of
  the synthetic 4k RPC camera): size-independent properties, and bf16 against the fp32 HIP
  path (which is parity-pinned) on the same rays and draws.
"""
import numpy as np
import pytest
import torch

import golden_util as gu
import spnerf_amd
from spnerf_amd import ReplayRandom, random_source
from test_gpu_bf16 import OUT_TOL
from test_gpu_parity import DEV, make_model

pytestmark = pytest.mark.gpu


def render_fixture(precision):
    data = gu.load("c5_w512")
    meta = data["meta"]
    dims, args = gu.dims_of(meta), gu.args_of(meta)
    assert args.n_samples == 128 and dims.sem and dims.width == 512 and meta["mode"] == "test"
    model = make_model(dims, meta["seed"], precision)
    with torch.no_grad(), random_source(ReplayRandom(gu.draws_of(data))) as src:
        res = spnerf_amd.render_rays({"coarse": model}, args, torch.tensor(data["rays"], device=DEV), None,
                                     semantics=torch.tensor(data["in_semantics"], device=DEV), mode="test")
    assert src.used == len(src.draws)
    return data, res


def test_c5_fixture_fp32_inference_matches_reference():
    data, res = render_fixture("fp32")
    keys = sorted(k[4:] for k in data if k.startswith("out_"))
    assert sorted(res) == keys
    for k in keys:
        gu.assert_close(k, res[k].cpu().numpy(), data["out_" + k], rtol=1e-4, atol_frac=1e-5)


def test_c5_fixture_bf16_inference_close_to_reference():
    data, res = render_fixture("bf16")
    errs = {}
    for k in sorted(k[4:] for k in data if k.startswith("out_")):
        got = res[k].cpu().numpy()
        assert np.isfinite(got).all(), k
        errs[k] = gu.rel_err(got, data["out_" + k])
    print({k: f"{v:.2e}" for k, v in errs.items()})
    assert max(errs.values()) < OUT_TOL, errs
    gu.assert_close("z_vals", res["z_vals_coarse"].cpu().numpy(), data["out_z_vals_coarse"], rtol=1e-6, atol_frac=1e-7)


class FixedU:
    """Stratified jitter from a given table; no σ noise (noise_std = 0)."""

    def __init__(self, u):
        self.u = u

    def rand(self, shape, device):
        assert tuple(shape) == tuple(self.u.shape)
        return self.u

    def noise(self, shape, device, noise_std):
        assert noise_std == 0
        return None


def test_c5_full_chunk_properties_and_bf16_vs_fp32():
    from spnerf_amd.satellite import image_rays, load_cameras
    cams = load_cameras()
    meta = cams["images"]["JAX_269_006_RGB"]
    ds = 0.2                                             # the x5 synthetic 4k camera of bench.py c5
    w = int(meta["width"] // ds)
    rays = image_rays(meta, ds, cams["scene_loc"], crop=(1600, 0, 32768 // w + 1, w), device=DEV)[:32768]
    B, S = rays.shape[0], 128
    assert B == 32768
    g = torch.Generator(device="cpu").manual_seed(0)
    sem = torch.randint(0, 3, (B,), generator=g).to(DEV)
    u = torch.rand(B, S, generator=g).to(DEV)
    args = gu.args_of({"args": dict(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.0, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    from oracle.weights import ModelDims
    dims = ModelDims(width=512, sem=True)
    out = {}
    for prec in ("fp32", "bf16"):
        model = make_model(dims, 4, prec)
        with torch.no_grad(), random_source(FixedU(u)):
            out[prec] = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sem, mode="test")
    r = out["bf16"]
    for k, v in r.items():
        assert torch.isfinite(v).all(), k
    z = r["z_vals_coarse"]
    assert torch.equal(z, out["fp32"]["z_vals_coarse"])
    assert bool((z[:, 1:] >= z[:, :-1]).all()) and bool((z >= rays[:, 6:7]).all()) and bool((z <= rays[:, 7:8]).all())
    wts, T = r["weights_coarse"], r["transparency_coarse"]
    assert bool((wts >= 0).all()) and bool((wts.sum(-1) <= 1 + 1e-5).all())
    assert bool((T[:, 1:] <= T[:, :-1] + 1e-7).all()) and bool((T[:, 0] == 1).all())
    # depth is a convex-ish combination of the sample depths: within [0, far]
    assert bool((r["depth_coarse"] >= 0).all()) and bool((r["depth_coarse"] <= rays[:, 7] * (1 + 1e-5) + 1e-7).all())
    rgb = r["rgb_coarse"]
    assert bool(((rgb >= 0) & (rgb <= 1)).all())
    for k in ("rgb_coarse", "depth_coarse", "sem_logits_coarse", "weights_coarse"):
        e = gu.rel_err(r[k].cpu().numpy(), out["fp32"][k].cpu().numpy())
        print(k, f"{e:.2e}")
        assert e < OUT_TOL, (k, e)


@pytest.mark.parametrize("sem", [True, False])
def test_fused_inference_heads_match_layer_by_layer_heads(sem):
    """bf16 inference with the fused heads kernel (σ, semantic hidden → logits, feat, Q, albedo,
    sun_v 2/3 → sun, sky on an LDS-resident 128-point tile; csrc/heads_bf16.hip) against the
    G / Q / sun_v GEMMs + k_heads_fwd_v path (option fused_heads=0) on the same rays and draws:
    same bf16 rounding points, other fp32 summation orders → norm-relative 2e-3 per key."""
    from spnerf_amd import _lib
    from oracle.weights import ModelDims
    g = torch.Generator(device="cpu").manual_seed(5)
    B, S = 3000, 128
    rays = torch.tensor(gu.synthetic_rays(B, 21), device=DEV)
    u = torch.rand(B, S, generator=g).to(DEV)
    labels = torch.randint(0, 3, (B,), generator=g).to(DEV)
    args = gu.args_of({"args": dict(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.0, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    model = make_model(ModelDims(width=512, sem=sem), 6, "bf16")
    outs = []
    try:
        for fused in (1, 0):
            _lib.set_option("fused_heads", fused)
            with torch.no_grad(), random_source(FixedU(u)):
                outs.append(spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=labels if sem else None,
                                                   mode="test"))
    finally:
        _lib.set_option("fused_heads", 1)
    for k in outs[1]:
        a, b = outs[0][k].cpu().numpy(), outs[1][k].cpu().numpy()
        assert np.isfinite(a).all(), k
        e = gu.rel_err(a, b)
        print(k, f"{e:.2e}")
        assert e < 2e-3, (k, e)


def test_inline_encoding_bit_identical():
    """The fused inference trunk encodes o + dir·z itself when it runs layer 0 (option pe_inline,
    no k_encode launch, no [P][64] fp32 PE round trip): the same pe_value arithmetic as k_encode,
    so every output is bit-identical to the k_encode path, with and without the semantic head."""
    from spnerf_amd import _lib
    from oracle.weights import ModelDims
    g = torch.Generator(device="cpu").manual_seed(9)
    B, S = 2000, 128
    rays = torch.tensor(gu.synthetic_rays(B, 23), device=DEV)
    u = torch.rand(B, S, generator=g).to(DEV)
    labels = torch.randint(0, 3, (B,), generator=g).to(DEV)
    args = gu.args_of({"args": dict(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.0, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    for sem in (True, False):
        model = make_model(ModelDims(width=512, sem=sem), 8, "bf16")
        outs = []
        try:
            for inline in (1, 0):
                _lib.set_option("pe_inline", inline)
                with torch.no_grad(), random_source(FixedU(u)):
                    outs.append(spnerf_amd.render_rays({"coarse": model}, args, rays, None,
                                                       semantics=labels if sem else None, mode="test"))
        finally:
            _lib.set_option("pe_inline", 1)
        for k in outs[1]:
            assert torch.equal(outs[0][k], outs[1][k]), (sem, k)


@pytest.mark.parametrize("th", [2, 1])
@pytest.mark.parametrize("sem,B,S", [(True, 3000, 128), (False, 301, 40), (True, 37, 128), (True, 300, 64)])
def test_trunk_with_fused_heads_bit_identical(sem, B, S, th):
    """The inference trunk running the fused heads on its last LDS image (option trunk_heads 2:
    the one-workgroup k_trunk_bf16<128> HEADS, the default; 1: k_trunk2_bf16 HEADS; H_L never goes
    to HBM) against the trunk launch followed by the heads kernel (trunk_heads 0, H_L through
    HBM): the same bf16 H_L bits and the same heads code (heads_tile.h), so every output is
    bit-identical.  301 x 40 points end in a ragged tile; 64 samples per ray put two rays' per-ray
    rows in one 128-point tile (trunk_heads 1 then falls back to the separate heads)."""
    from spnerf_amd import _lib
    from oracle.weights import ModelDims
    g = torch.Generator(device="cpu").manual_seed(11)
    rays = torch.tensor(gu.synthetic_rays(B, 25), device=DEV)
    u = torch.rand(B, S, generator=g).to(DEV)
    labels = torch.randint(0, 3, (B,), generator=g).to(DEV)
    args = gu.args_of({"args": dict(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.0, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    model = make_model(ModelDims(width=512, sem=sem), 9, "bf16")
    outs = []
    if th == 1 and not _lib.has_option("trunk2"):
        pytest.skip("trunk_heads 1 rides on the two-workgroup trunk k_trunk2_bf16 (ablation build only)")
    try:
        for t in (th, 0):
            _lib.set_option("trunk_heads", t)
            if th == 1:
                _lib.set_option("trunk2", 3 if t == 1 else 0)
            with torch.no_grad(), random_source(FixedU(u)):
                outs.append(spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=labels if sem else None,
                                                   mode="test"))
    finally:
        _lib.set_option("trunk_heads", 2)
        if th == 1:
            _lib.set_option("trunk2", 0)
    for k in outs[1]:
        assert torch.isfinite(outs[0][k]).all(), k
        assert torch.equal(outs[0][k], outs[1][k]), (k, float((outs[0][k] - outs[1][k]).abs().max()))


@pytest.mark.parametrize("sem", [True, False])
def test_fused_inference_kernel_vs_layer_by_layer_gemms(sem):
    """The product C5 kernel (k_trunk_bf16<128, 4096>: trunk + heads in one launch, the default)
    against the product library's layer-by-layer path (fused_trunk 0, trunk_heads 0: layer 0 on
    the hi/lo-plane k_gemm_nt_bf16 after k_encode, layers 1..7 one bf16 GEMM each with the sine
    epilogue, then the heads kernel) on 3 000 rays x 128 samples: other kernels and tilings over
    the same bf16 rounding points, the same k order and the same epilogue arithmetic, so every
    output is bit-identical (measured so on MI355X, profiles/r06/gpu_suite.txt)."""
    from spnerf_amd import _lib
    from oracle.weights import ModelDims
    g = torch.Generator(device="cpu").manual_seed(13)
    B, S = 3000, 128
    rays = torch.tensor(gu.synthetic_rays(B, 27), device=DEV)
    u = torch.rand(B, S, generator=g).to(DEV)
    labels = torch.randint(0, 3, (B,), generator=g).to(DEV)
    args = gu.args_of({"args": dict(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                    sc_lambda=0.0, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    model = make_model(ModelDims(width=512, sem=sem), 10, "bf16")
    outs = []
    try:
        for fused in (1, 0):
            _lib.set_option("fused_trunk", fused)
            _lib.set_option("trunk_heads", 2 if fused else 0)
            with torch.no_grad(), random_source(FixedU(u)):
                outs.append(spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=labels if sem else None,
                                                   mode="test"))
    finally:
        _lib.set_option("fused_trunk", 1)
        _lib.set_option("trunk_heads", 2)
    for k in outs[1]:
        a, b = outs[0][k].cpu().numpy(), outs[1][k].cpu().numpy()
        assert np.isfinite(a).all() and np.isfinite(b).all(), k
        e = gu.rel_err(a, b)
        print(k, f"norm-rel {e:.2e} max-abs {float(np.abs(a - b).max()):.2e} bitwise {np.array_equal(a, b)}")
        assert np.array_equal(a, b), (k, e)
