"""Fused bf16 trunk (k_trunk_bf16: fc_net layers 1..L-1 in one persistent launch, activations
resident in LDS) vs the layer-by-layer bf16 GEMMs it replaces — needs an MI355X.

Both paths do the same arithmetic in the same k-order (fp32 accumulation of the same bf16
products, the same epilogue), so renders and gradients must agree bit for bit (measured: they
do); the bf16 path itself is held to the reference by tests/test_gpu_bf16.py.  Covered: the guided-sampling
pass 1 (no saved activations, sigma only), pass 2 and the solar pass (saved H / D feeding the
backward), the skip layer's PE columns and per-ray semantic rows, point counts that are not a
multiple of the 128-point tile, and PE off (K0p = 32).  fc_net.0 runs on bf16 hi/lo planes
(l0_split): inside the fused launch when nothing is saved (the point network below; also when
saving with trunk_l0=2), as a separate GEMM otherwise, with the same planes and k-order.
"""
import numpy as np
import pytest
import torch

import golden_util as gu
import spnerf_amd
from spnerf_amd import _lib
from oracle.weights import ModelDims
from test_gpu_parity import DEV, gu_rays, make_model

pytestmark = pytest.mark.gpu
TOL = 1e-5  # norm-relative


def _render(fused: bool, dims: ModelDims, n_rays: int, guided: bool, sc: float, seed: int = 0, n_samples: int = 64,
            options: dict | None = None):
    # (heads_epi 0: the narrow heads on k_heads_fwd_v for every variant compared here — the epilogue
    # heads need the trunk's σ column, which not every trunk variant writes)
    opts = {"fused_trunk": int(fused), "heads_epi": 0, **(options or {})}
    saved = {k: _lib.get_option(k) for k in opts}
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        args = gu.args_of({"args": dict(n_samples=n_samples, n_importance=0, model="sp-nerf", beta=False, guidedsample=guided,
                                        sc_lambda=sc, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
        rays = torch.tensor(gu_rays(n_rays, 9 + seed), device=DEV)
        g = torch.Generator(device="cpu").manual_seed(seed)
        kw = {}
        if guided:
            kw = dict(valid_depth=(torch.rand(n_rays, generator=g) < 0.68).long().to(DEV),
                      target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n_rays, device=DEV)], 1),
                      target_std=torch.full((n_rays,), 0.01, device=DEV))
        sem = torch.randint(-1, 3, (n_rays,), generator=g).to(DEV) if dims.sem else None
        if sem is not None:
            sem = torch.where(sem < 0, torch.full_like(sem, -100), sem)
        model = make_model(dims, 2, "bf16")
        torch.manual_seed(123)  # same device draws for both runs
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sem, mode="train", **kw)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        loss.backward()
        torch.cuda.synchronize()
        return ({k: v.detach().cpu() for k, v in res.items()},
                {n: p.grad.detach().cpu() for n, p in model.named_parameters() if p.grad is not None})
    finally:
        for k, v in saved.items():
            _lib.set_option(k, v)


def _assert_bitwise(a, b):
    (r1, g1), (r0, g0) = a, b
    assert sorted(r1) == sorted(r0) and sorted(g1) == sorted(g0)
    for k in r0:
        assert torch.isfinite(r1[k]).all(), k
        assert torch.equal(r1[k], r0[k]), (k, gu.rel_err(r1[k].numpy(), r0[k].numpy()))
    for n in g0:
        assert torch.equal(g1[n], g0[n]), (n, gu.rel_err(g1[n].numpy(), g0[n].numpy()))


@pytest.mark.parametrize("dims,n_rays,guided,sc", [
    (ModelDims(width=512, sem=True), 257, True, 0.1),     # C3 flags; 257·64 points: ragged last tile
    (ModelDims(width=512), 1024, False, 0.0),             # C2 flags at bf16
    (ModelDims(width=512, mapping=False), 130, False, 0.1),  # no PE: K0p = 32 skip columns
])
def test_fused_trunk_matches_layerwise(dims, n_rays, guided, sc):
    assert _lib.get_option("fused_trunk") == 1
    r1, g1 = _render(True, dims, n_rays, guided, sc)
    r0, g0 = _render(False, dims, n_rays, guided, sc)
    assert sorted(r1) == sorted(r0) and sorted(g1) == sorted(g0)
    same = True
    for k in r0:
        assert torch.isfinite(r1[k]).all(), k
        e = gu.rel_err(r1[k].numpy(), r0[k].numpy())
        same &= torch.equal(r1[k], r0[k])
        assert e <= TOL, (k, e)
    worst = 0.0
    for n in g0:
        e = gu.rel_err(g1[n].numpy(), g0[n].numpy()) if g0[n].abs().sum() > 0 else float(g1[n].abs().sum())
        same &= torch.equal(g1[n], g0[n])
        worst = max(worst, e)
        assert e <= TOL, (n, e)
    print(f"fused vs layer-by-layer: bitwise={same} worst grad rel err {worst:.2e}")
    assert same


def test_fused_trunk_with_layer0_when_saving_bitwise_vs_layerwise():
    """trunk_l0=2 (the default): fc_net.0 inside the fused launch also when activations are saved
    (the training tiles, D = w0·cos(w0·z) of layer 0 from the trunk's epilogue); trunk_l0=1 keeps it a
    separate GEMM there."""
    old = _lib.get_option("trunk_l0")
    try:
        for l0 in (1, 2):   # the separate layer-0 GEMM when saving, and layer 0 inside the launch
            _lib.set_option("trunk_l0", l0)
            test_fused_trunk_matches_layerwise(ModelDims(width=512, sem=True), 257, True, 0.1)
    finally:
        _lib.set_option("trunk_l0", old)


def test_fused_trunk_point_network_bitwise_vs_layerwise():
    """SPNeRF.forward on 3000 points (S = 1: every point its own ray, semantic + beta heads)."""
    dims = ModelDims(width=512, sem=True, beta=True)
    rng = np.random.default_rng(5)
    P = 3000
    xyz = torch.tensor(rng.uniform(-1, 1, (P, 3)).astype(np.float32), device=DEV)
    sun = torch.tensor(rng.normal(size=(P, 3)).astype(np.float32), device=DEV)
    lab = torch.tensor(rng.choice([0, 1, 2, -100], size=P).astype(np.int64), device=DEV)
    t = torch.tensor(rng.normal(size=(P, dims.t_dim)).astype(np.float32), device=DEV)
    m = make_model(dims, 4, "bf16")
    outs = []
    for fused in (1, 0):
        _lib.set_option("fused_trunk", fused)
        try:
            with torch.no_grad():
                outs.append(m(xyz, input_sun_dir=sun, input_t=t, input_s=lab).cpu())
        finally:
            _lib.set_option("fused_trunk", 1)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dims,n_rays,guided,sc,n_samples", [
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64),   # C3 flags: semantic rows at the skip layer
    (ModelDims(width=512), 33, False, 0.1, 32),             # 33·32 points: the last 64-point tile half full
    (ModelDims(width=512, sem=True), 96, False, 0.0, 128),  # C5-like sampling, semantic rows
])
def test_two_workgroup_trunk_bitwise(dims, n_rays, guided, sc, n_samples):
    """k_trunk2_bf16 (D stored from the registers, trunk2_bf16.hip; 128-point tiles, or 64-point
    tiles two workgroups per CU) against the one-workgroup kernels with the D image: training
    (trunk2=1), training and inference (trunk2=2, layer 0 and the inline encoding in the launch)
    and inference only (trunk2=3) equal trunk2=0 (the default) bit for bit."""
    base = _render(True, dims, n_rays, guided, sc, n_samples=n_samples, options={"trunk2": 0})
    for tile in (128, 64):
        for t2 in (1, 2, 3):
            _assert_bitwise(_render(True, dims, n_rays, guided, sc, n_samples=n_samples,
                                    options={"trunk2": t2, "trunk2_tile": tile}), base)


@pytest.mark.parametrize("dims,n_rays,guided,sc,n_samples,l0", [
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64, 1),  # C3 flags: the skip layer keeps the D image
    (ModelDims(width=512), 33, False, 0.1, 32, 1),            # the last 64-point tile half full
    (ModelDims(width=512), 40, False, 0.0, 64, 2),            # layer 0 in the launch (w0 = 30, no rows)
])
def test_training_trunk_register_d_bitwise(dims, n_rays, guided, sc, n_samples, l0):
    """k_trunk_bf16<64> with D = cos stored from the accumulators during the epilogue (option
    trunk_dreg 1, the default; layers with per-ray rows keep the D image) against the D image
    drained behind the next k-loop (0): the same values, so renders and gradients bit for bit."""
    opts = {"trunk_l0": l0, "trunk_tile": 64}
    base = _render(True, dims, n_rays, guided, sc, n_samples=n_samples, options=dict(opts, trunk_dreg=0))
    _assert_bitwise(_render(True, dims, n_rays, guided, sc, n_samples=n_samples, options=dict(opts, trunk_dreg=1)), base)


@pytest.mark.parametrize("dims,n_rays,guided,sc,n_samples,l0", [
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64, 2),  # C3 flags, layer 0 in the launch
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64, 1),  # layer 0 as its own GEMM
    (ModelDims(width=512), 33, False, 0.1, 32, 2),            # 33·32 points: the last 128-point tile a quarter full
])
def test_training_trunk_128_point_tiles_bitwise(dims, n_rays, guided, sc, n_samples, l0):
    """The training trunk on 128-point tiles (option trunk_tile 128: cos through the image
    between two barriers, then sin; σ pre-activation rows from the last image) against the
    64-point tiles: the same per-point arithmetic and k order, so renders and gradients bit for
    bit, with the narrow heads on k_heads_fwd_v and in the head GEMMs' epilogues."""
    for hepi in (0, 1):
        opts = {"trunk_l0": l0, "heads_epi": hepi}
        base = _render(True, dims, n_rays, guided, sc, n_samples=n_samples, options=dict(opts, trunk_tile=64))
        _assert_bitwise(_render(True, dims, n_rays, guided, sc, n_samples=n_samples, options=dict(opts, trunk_tile=128)), base)


@pytest.mark.parametrize("tile", [64, 128])
@pytest.mark.parametrize("dims,n_rays,guided,sc,n_samples", [
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64),   # C3 flags: main (all heads) and solar (σ + sun) passes
    (ModelDims(width=512), 33, False, 0.1, 32),             # the last tile partly full
])
def test_training_trunk_sigma_rows_bitwise(dims, n_rays, guided, sc, n_samples, tile):
    """The training trunk writing each point's σ pre-activation from its last layer's LDS image
    (option trunk_sigma 1, the default: k_heads_fwd_v's lane layout, dot4 order and wave_total, so
    the wave-per-point heads skip H_L) against the heads computing it from H_L (0): renders and
    gradients bit for bit."""
    base = _render(True, dims, n_rays, guided, sc, n_samples=n_samples, options={"trunk_sigma": 0, "trunk_tile": tile})
    _assert_bitwise(_render(True, dims, n_rays, guided, sc, n_samples=n_samples, options={"trunk_sigma": 1, "trunk_tile": tile}), base)


@pytest.mark.parametrize("dims,n_rays,guided,sc,n_samples", [
    (ModelDims(width=512, sem=True), 257, True, 0.1, 64),   # C3 flags: main + solar passes (sun directions)
    (ModelDims(width=512), 33, False, 0.1, 32),             # ragged last tile
])
def test_training_trunk_inline_encoding_bitwise(dims, n_rays, guided, sc, n_samples):
    """Training forwards with layer 0 in the trunk encode o + dir·z in the trunk's staging (option
    pe_inline 1, the default: no k_encode launch, no fp32 [P][64] PE round trip; the trunk writes
    the bf16 PE rows X0b the weight gradients read) against k_encode (pe_inline 0): the same
    pe_value arithmetic, so renders and gradients bit for bit."""
    base = _render(True, dims, n_rays, guided, sc, n_samples=n_samples, options={"pe_inline": 0})
    _assert_bitwise(_render(True, dims, n_rays, guided, sc, n_samples=n_samples, options={"pe_inline": 1}), base)
