"""fp32 GEMM kernel variants through a whole training render — needs an MI355X.

Every fp32 NT variant (`nt_f32_variant` 5 … 8: register staging one / two K-steps ahead, LDS-DMA
on one 8-wave block or on two 4-wave blocks per CU) and TN variant (`tn_f32_variant` 0 … 2)
accumulates each output in the same k-order, so a C2-shaped render (W = 512, semantic and sun
heads on, guided pass) and its parameter gradients must come out bit for bit the same as with
the defaults; the defaults themselves are held to the reference by tests/test_gpu_parity.py.
"""
import pytest
import torch

import golden_util as gu
import spnerf_amd
from spnerf_amd import _lib
from oracle.weights import ModelDims
from test_gpu_parity import DEV, gu_rays, make_model

pytestmark = pytest.mark.gpu


def _render(opts):
    old = {k: _lib.get_option(k) for k in opts}
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                        sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
        n = 300  # 300 · 64 points: ragged last tiles for every tiling
        rays = torch.tensor(gu_rays(n, 21), device=DEV)
        g = torch.Generator(device="cpu").manual_seed(4)
        kw = dict(valid_depth=(torch.rand(n, generator=g) < 0.7).long().to(DEV),
                  target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n, device=DEV)], 1),
                  target_std=torch.full((n,), 0.01, device=DEV))
        sem = torch.randint(0, 3, (n,), generator=g).to(DEV)
        model = make_model(ModelDims(width=512, sem=True), 6, "fp32")
        torch.manual_seed(7)
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sem, mode="train", **kw)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        loss.backward()
        torch.cuda.synchronize()
        return ({k: v.detach().cpu() for k, v in res.items()},
                {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


@pytest.mark.parametrize("opts", [{"nt_f32_variant": v} for v in (5, 6, 7, 8)] +
                         [{"tn_f32_variant": v} for v in (0, 1, 2)])
def test_fp32_gemm_variants_bitwise_equal(opts):
    r0, g0 = _render({})
    r1, g1 = _render(opts)
    assert sorted(r0) == sorted(r1) and sorted(g0) == sorted(g1)
    for k in r0:
        assert torch.isfinite(r0[k]).all(), k
        assert torch.equal(r0[k], r1[k]), (opts, k)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), (opts, k)


def _render_bf16(opts, n=300, ns=64):
    opts = {"heads_epi": 0, **opts}   # (k_heads_fwd_v for every GEMM variant compared: see test_gpu_trunk._render)
    old = {k: _lib.get_option(k) for k in opts}
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        args = gu.args_of({"args": dict(n_samples=ns, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                        sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
        rays = torch.tensor(gu_rays(n, 22), device=DEV)
        g = torch.Generator(device="cpu").manual_seed(5)
        kw = dict(valid_depth=(torch.rand(n, generator=g) < 0.7).long().to(DEV),
                  target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n, device=DEV)], 1),
                  target_std=torch.full((n,), 0.01, device=DEV))
        sem = torch.randint(0, 3, (n,), generator=g).to(DEV)
        model = make_model(ModelDims(width=512, sem=True), 6, "bf16")
        torch.manual_seed(7)
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sem, mode="train", **kw)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        loss.backward()
        torch.cuda.synchronize()
        return ({k: v.detach().cpu() for k, v in res.items()},
                {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


@pytest.mark.parametrize("variant", [2, 3])
def test_bf16_tn_tilings_agree(variant):
    """bf16 weight gradients: the 256x256 TN tilings (tn_bf16_variant 2: register-staged, 3:
    LDS-DMA; one block per CU) against the 128x128 one (1).  They split the points differently, so the fp32 slab sums round
    differently: renders must be bit-identical (the TN GEMMs only feed gradients) and every
    gradient within 1e-4 of its largest entry — fp32 summation-order noise, far below the bf16
    operand rounding both share."""
    r1, g1 = _render_bf16({"tn_bf16_variant": 1})
    r2, g2 = _render_bf16({"tn_bf16_variant": variant})
    for k in r1:
        assert torch.equal(r1[k], r2[k]), k
    assert sorted(g1) == sorted(g2)
    for k in g1:
        assert torch.isfinite(g2[k]).all(), k
        scale = g1[k].abs().max().item()
        assert (g1[k] - g2[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


def test_bf16_skip_layer_tail_split_agrees():
    """The skip layer's weight gradient ([H | x0], K = 512 + K0p) at >= 2^18 points runs as the
    wide K = 512 GEMM plus the K0p tail (option tn_split_tail): gradients within 1e-4 of the
    single-launch 128x128 tiling's (different point splits: fp32 summation-order noise), renders
    bit-identical."""
    r1, g1 = _render_bf16({"tn_split_tail": 0}, n=2048)
    r2, g2 = _render_bf16({"tn_split_tail": 1}, n=2048)
    for k in r1:
        assert torch.equal(r1[k], r2[k]), k
    for k in g1:
        scale = g1[k].abs().max().item()
        assert (g1[k] - g2[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


@pytest.mark.parametrize("n,ns", [(300, 64), (301, 40), (1, 16)])
def test_bf16_fused_backward_bitwise_equal(n, ns):
    """The fused backward dX chain (k_trunk_bwd_bf16, option fused_bwd) multiplies each layer's
    fp32 accumulator by D over the same k order as the layer-by-layer x Dmul GEMMs: every dZ, so
    every gradient, is bit-identical.  301 x 80 points leave a ragged last 64-point tile; one ray of
    32 points is a single, half-empty tile."""
    r0, g0 = _render_bf16({"fused_bwd": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"fused_bwd": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("opts,n,ns", [({"nt_bf16_epi": 0}, 300, 64), ({"nt_bf16_epi": 0}, 301, 40),
                                       ({"nt_bf16_variant": 5}, 300, 64)])
def test_bf16_nt_epilogue_variants_bitwise_equal(opts, n, ns):
    """The DMA NT GEMM's compile-time epilogue variants (bias + sine; + per-ray rows read once per
    tile and spread by ds_bpermute; rank-1 + Dmul; stores through buffer descriptors) against the
    generic runtime-flag epilogue (nt_bf16_epi 0) and the register-staged kernel (nt_bf16_variant
    5): same arithmetic, same k order — renders and gradients bit for bit.  40 samples per ray (80
    after the guided pass) is not a multiple of 32 rows: the per-ray-row variant falls back."""
    r0, g0 = _render_bf16({}, n=n, ns=ns)
    r1, g1 = _render_bf16(opts, n=n, ns=ns)
    for k in r0:
        assert torch.isfinite(r0[k]).all(), k
        assert torch.equal(r0[k], r1[k]), (opts, k)
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), (opts, k)


@pytest.mark.parametrize("n,ns", [(300, 64), (301, 40)])
def test_bf16_tile_rowsum_agrees(n, ns):
    """The per-ray sums of dZ_0 / dZ_skip (the semantic columns' gradients) by 64-point tiles —
    formed from the fused dX chain's LDS image (option tile_rowsum 1) — against the per-ray
    k_ray_rowsum16 over HBM (0): a different fp32 summation order, so gradients agree to 1e-4 of
    their largest entry and renders bit for bit; 40 + 40 samples per ray is not a whole number of
    tiles (falls back to the per-ray sums: bit-identical)."""
    r0, g0 = _render_bf16({"tile_rowsum": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"tile_rowsum": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        assert (g0[k] - g1[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k
        if ns % 64:
            assert torch.equal(g0[k], g1[k]), k


def test_bf16_tn_bias_split_agrees():
    """The DMA weight-gradient GEMM's bias sums split over the two k-tiles of each column range
    (option tn_bf16_bias_split 1, so partner tiles do equal work and share the A rows in L2)
    against the whole bias on the k0 = 0 tile (0): another fp32 order of the same bf16 sums —
    gradients within 1e-4 of their largest entry, renders bit for bit.  2 048 rays: the
    256x256 DMA tiling runs."""
    r0, g0 = _render_bf16({"tn_bf16_bias_split": 0}, n=2048)
    r1, g1 = _render_bf16({"tn_bf16_bias_split": 1}, n=2048)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        assert (g0[k] - g1[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


@pytest.mark.parametrize("n", [300, 2048])
def test_bf16_tn_few_tiles_agrees(n):
    """Weight gradients of 256-wide layers (sun_v_net.2 / .4, the solar pass's sun_v_net.0) on
    the 256x256 DMA tiling with more point splits (option tn_bf16_few_tiles 1) against the
    128x128 tiling (0): other point splits, so fp32 slab sums round differently — gradients within
    1e-4 of their largest entry, renders bit for bit."""
    r0, g0 = _render_bf16({"tn_bf16_few_tiles": 0}, n=n)
    r1, g1 = _render_bf16({"tn_bf16_few_tiles": 1}, n=n)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        assert (g0[k] - g1[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


@pytest.mark.parametrize("n,ns", [(300, 64), (2048, 64), (301, 40)])
def test_bf16_tn_k64_agrees(n, ns):
    """fc_net.0's weight gradient and the skip layer's PE tail (N = 512, K = 64) on the narrow
    kernel holding the whole 512 x 64 output per split (option tn_bf16_k64 1; the skip layer's tail
    runs on it at >= 2^18 points: 2 048 x 128) against the 128x128 tiling (0):
    other point splits and summation order — gradients within 1e-4 of their largest entry,
    renders bit for bit.  300 x 128 and 301 x 80 points leave a ragged last split."""
    r0, g0 = _render_bf16({"tn_bf16_k64": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"tn_bf16_k64": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        assert (g0[k] - g1[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


@pytest.mark.parametrize("n,ns", [(300, 64), (301, 40), (1, 16)])
def test_bf16_fused_backward_register_dz_bitwise_equal(n, ns):
    """The fused dX chain storing each dZ from its epilogue's registers (option trunk_bwd_dreg 1;
    measured slower, off by default) against the copy-out from the LDS image behind the next
    k-loop (0, the default): the same
    values in the same rows — renders and gradients bit for bit (ragged and half-empty tiles)."""
    r0, g0 = _render_bf16({"trunk_bwd_dreg": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"trunk_bwd_dreg": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        assert torch.equal(g0[k], g1[k]), k



@pytest.mark.parametrize("n,ns", [(300, 64), (2048, 64)])
def test_bf16_tn_prefetched_fragments_bitwise_equal(n, ns):
    """Option tn_bf16_pf: the DMA weight-gradient GEMM reading the next k-step's LDS fragments
    during the current k-step's MFMAs (same MFMAs, same order) gives the same gradients bit for bit
    — per-pass launches here, the deferred group launches below."""
    r0, g0 = _render_bf16({"tn_bf16_pf": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"tn_bf16_pf": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    assert sorted(g0) == sorted(g1)
    for k in g0:
        assert torch.isfinite(g0[k]).all(), k
        assert torch.equal(g0[k], g1[k]), k


def test_bf16_tn_prefetched_fragments_grouped_bitwise_equal():
    from test_gpu_flatgrad import _deferred_grads
    old = _lib.get_option("tn_bf16_pf")
    out = []
    try:
        for pf in (0, 1):
            _lib.set_option("tn_bf16_pf", pf)
            out.append(_deferred_grads(9, n_rays=256)[0])
    finally:
        _lib.set_option("tn_bf16_pf", old)
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


@pytest.mark.parametrize("n,ns", [(300, 64), (2048, 64)])
def test_bf16_tn_quad_wave_bitwise_equal(n, ns):
    """Option tn_bf16_quad: the 4-wave (128x128 per wave) DMA weight-gradient kernel keeps every
    output's k-order and the bias sums' phase order: gradients bit for bit equal."""
    r0, g0 = _render_bf16({"tn_bf16_quad": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"tn_bf16_quad": 1}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    for k in g0:
        assert torch.isfinite(g0[k]).all(), k
        assert torch.equal(g0[k], g1[k]), k


def test_bf16_tn_quad_wave_grouped_bitwise_equal():
    from test_gpu_flatgrad import _deferred_grads
    old = _lib.get_option("tn_bf16_quad")
    out = []
    try:
        for q in (0, 1):
            _lib.set_option("tn_bf16_quad", q)
            out.append(_deferred_grads(9, n_rays=256)[0])
    finally:
        _lib.set_option("tn_bf16_quad", old)
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_bf16_nt_dma_issue_placement_bitwise_equal():
    """Options nt_bf16_ip / nt_bf16_ip_gen (ablation build): the head and dX GEMMs issuing the next
    DMA step one instruction per two MFMA groups (3) instead of between the k-halves (2, the
    default) change no MFMA and no order — renders and gradients bit for bit, the heads in the GEMM
    epilogues included."""
    r0, g0 = _render_bf16({"heads_epi": 1, "nt_bf16_ip": 2, "nt_bf16_ip_gen": 2}, n=2048, ns=64)
    r1, g1 = _render_bf16({"heads_epi": 1, "nt_bf16_ip": 3, "nt_bf16_ip_gen": 3}, n=2048, ns=64)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


def _close_or_equal(a, b, bitwise, k):
    if bitwise:
        assert torch.equal(a, b), k
    else:
        assert torch.isfinite(b).all(), k
        err = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30)
        assert err <= 1e-5, (k, err)


@pytest.mark.parametrize("ip", [2, 3, 4, 5])
def test_bf16_tn_dma_issue_placement_bitwise_equal(ip):
    """Option tn_bf16_ip (ablation build): where the weight-gradient GEMM issues the next DMA
    step (2: between its k-halves, 3: one instruction per two MFMA groups) changes no MFMA and no
    order — gradients bit for bit equal to the default placement, per pass and grouped; 4 (the two
    waves of a SIMD a k-step apart) and 5 (the default schedule) sum the biases from the fragments
    in registers — another fixed order: weight gradients bitwise, biases within 1e-5."""
    from test_gpu_flatgrad import _deferred_grads
    r0, g0 = _render_bf16({"tn_bf16_ip": 1}, n=2048, ns=64)
    r1, g1 = _render_bf16({"tn_bf16_ip": ip}, n=2048, ns=64)
    for k in g0:
        _close_or_equal(g0[k], g1[k], ip < 4 or not k.endswith("bias"), k)
    old = _lib.get_option("tn_bf16_ip")
    out = []
    try:
        for v in (1, ip):
            _lib.set_option("tn_bf16_ip", v)
            out.append(_deferred_grads(9, n_rays=256)[0])
    finally:
        _lib.set_option("tn_bf16_ip", old)
    for k in out[0]:
        _close_or_equal(out[0][k], out[1][k], ip < 4 or not k.endswith("bias"), k)


@pytest.mark.parametrize("m16", [1, 2, 3, 4])
@pytest.mark.parametrize("n,ns", [(300, 64), (2048, 64)])
def test_bf16_tn_m16_agrees(m16, n, ns):
    """Option tn_bf16_m16: the weight gradients on 16x16x32 MFMAs (32-point blocks per output
    element; 4 or 5 DMA stages) against the 32x32x16 kernel: renders bit for bit, every gradient
    within 1e-5 of its largest entry (fp32 sums of the same bf16 products in another grouping)."""
    r0, g0 = _render_bf16({"tn_bf16_m16": 0}, n=n, ns=ns)
    r1, g1 = _render_bf16({"tn_bf16_m16": m16}, n=n, ns=ns)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        err = (g0[k] - g1[k]).abs().max().item() / max(g0[k].abs().max().item(), 1e-30)
        assert err <= 1e-5, (k, err)


def test_bf16_tn_m16_grouped_agrees():
    from test_gpu_flatgrad import _deferred_grads
    old = _lib.get_option("tn_bf16_m16")
    out = []
    try:
        for m in (0, 1, 3):
            _lib.set_option("tn_bf16_m16", m)
            out.append(_deferred_grads(9, n_rays=256)[0])
    finally:
        _lib.set_option("tn_bf16_m16", old)
    for o in out[1:]:
        for k in out[0]:
            err = (out[0][k] - o[k]).abs().max().item() / max(out[0][k].abs().max().item(), 1e-30)
            assert err <= 1e-5, (k, err)


def test_pack_table_bitwise_equal():
    """Option pack_table: the weight re-pack from a device-resident piece table (one launch)
    writes the same packed buffer as the kernarg-table launches (two for the bf16 MLP)."""
    model = make_model(ModelDims(width=512, sem=True, beta=True), 3, "bf16")
    old = _lib.get_option("pack_table")
    bufs, launches = [], []
    try:
        for t in (0, 1):
            _lib.set_option("pack_table", t)
            model.packed_weights()          # (first use builds the table)
            torch.cuda.synchronize()
            _lib.prof_reset()
            _lib.prof_enable(True)
            bufs.append(model.packed_weights().clone())
            torch.cuda.synchronize()
            _lib.prof_enable(False)
            launches.append(_lib.prof_read("pack")["launches"])
    finally:
        _lib.set_option("pack_table", old)
    assert torch.equal(bufs[0], bufs[1])
    assert launches == [2, 1], launches


def _render_heads(opts, beta, n=300):
    """A C3-flag bf16 training render (guided 64 + 64 samples, solar pass, semantic head; beta
    with a t embedding) and its gradients under library options."""
    old = {k: _lib.get_option(k) for k in opts}
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=beta, guidedsample=True,
                                        sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
        rays = torch.tensor(gu_rays(n, 23), device=DEV)
        g = torch.Generator(device="cpu").manual_seed(6)
        kw = dict(valid_depth=(torch.rand(n, generator=g) < 0.7).long().to(DEV),
                  target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n, device=DEV)], 1),
                  target_std=torch.full((n,), 0.01, device=DEV))
        sem = torch.randint(0, 3, (n,), generator=g).to(DEV)
        model = make_model(ModelDims(width=512, sem=True, beta=beta), 6, "bf16")
        models = {"coarse": model}
        ts = None
        if beta:
            torch.manual_seed(1)
            models["t"] = torch.nn.Embedding(4, model.t_embedding_dims).to(DEV)
            ts = torch.randint(0, 4, (n,), generator=g).to(DEV)
        torch.manual_seed(7)
        res = spnerf_amd.render_rays(models, args, rays, ts, semantics=sem, mode="train", **kw)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        loss.backward()
        torch.cuda.synchronize()
        return ({k: v.detach().cpu() for k, v in res.items()},
                {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


@pytest.mark.parametrize("beta", [False, True])
def test_heads_in_gemm_epilogue_agree(beta):
    """Option heads_epi: the narrow heads (rgb, sun, beta, semantic logits; σ and sky with the sun)
    computed in the epilogues of the G / Q / sun_v.3 GEMMs instead of k_heads_fwd_v: the same
    dot products over the same bf16 inputs in another fp32 summation order — renders and gradients
    agree to fp32 rounding."""
    r0, g0 = _render_heads({"heads_epi": 0}, beta)
    r1, g1 = _render_heads({"heads_epi": 1}, beta)
    assert sorted(r0) == sorted(r1) and sorted(g0) == sorted(g1)
    for k in r0:
        assert torch.isfinite(r1[k]).all(), k
        scale = r0[k].abs().max().item()
        assert (r0[k] - r1[k]).abs().max().item() <= 1e-5 * scale + 1e-7, k
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        assert (g0[k] - g1[k]).abs().max().item() <= 1e-4 * scale + 1e-30, k


def _render_train_heads(opts, sem, n, n_samples, guided, precision="bf16"):
    """A bf16 training render (solar pass on, semantic head optional) and its gradients."""
    old = {k: _lib.get_option(k) for k in opts}
    for k, v in opts.items():
        _lib.set_option(k, v)
    try:
        args = gu.args_of({"args": dict(n_samples=n_samples, n_importance=0, model="sp-nerf", beta=False,
                                        guidedsample=guided, sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120,
                                        noise_std=0.0)})
        rays = torch.tensor(gu_rays(n, 31), device=DEV)
        g = torch.Generator(device="cpu").manual_seed(8)
        kw = {}
        if guided:
            kw = dict(valid_depth=(torch.rand(n, generator=g) < 0.7).long().to(DEV),
                      target_depths=torch.stack([rays[:, 7] * 0.5, torch.ones(n, device=DEV)], 1),
                      target_std=torch.full((n,), 0.01, device=DEV))
        labels = torch.randint(0, 3, (n,), generator=g).to(DEV) if sem else None
        model = make_model(ModelDims(width=512, sem=sem), 9, precision)
        torch.manual_seed(7)
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=labels, mode="train", **kw)
        loss = sum((v.float() ** 2).mean() for k, v in sorted(res.items()) if v.requires_grad)
        loss.backward()
        torch.cuda.synchronize()
        return ({k: v.detach().cpu() for k, v in res.items()},
                {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


@pytest.mark.parametrize("sem,n,n_samples,guided", [(True, 300, 64, True), (False, 97, 40, False), (True, 97, 40, False)])
def test_training_heads_kernel_agree(sem, n, n_samples, guided):
    """Option heads_epi 2: the training heads (G, Q, sun_v 2 / 3 with every saved activation, and
    the narrow heads) in one LDS-resident launch after the saving trunk, main and solar pass.
    The wide layers are the layer-by-layer GEMMs' arithmetic, so what the backward reads from them
    is the same; the narrow heads sum in another fp32 order (MFMA instead of the GEMM epilogues /
    k_heads_fwd_v): renders and gradients agree to fp32 rounding.  97 rays x 40 samples: a ragged
    last tile, and a sample count the epilogue heads do not take (their fallback is the reference)."""
    r0, g0 = _render_train_heads({"heads_epi": 1}, sem, n, n_samples, guided)
    r1, g1 = _render_train_heads({"heads_epi": 2}, sem, n, n_samples, guided)
    assert sorted(r0) == sorted(r1) and sorted(g0) == sorted(g1)
    for k in r0:
        assert torch.isfinite(r1[k]).all(), k
        scale = r0[k].abs().max().item()
        assert (r0[k] - r1[k]).abs().max().item() <= 1e-5 * scale + 1e-7, k
    # (the narrow heads' weights ride as bf16 hi + lo rows, ~2^-17 relative, as in the inference
    # heads: per tensor within 5e-4 of its largest entry, the whole gradient within 1e-4)
    worst, num, den = {}, 0.0, 0.0
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        scale = g0[k].abs().max().item()
        worst[k] = (g0[k] - g1[k]).abs().max().item() / (scale + 1e-30)
        num += float(((g0[k] - g1[k]).double() ** 2).sum())
        den += float((g0[k].double() ** 2).sum())
    print({k: f"{v:.1e}" for k, v in sorted(worst.items(), key=lambda x: -x[1])[:6]}, (num / den) ** 0.5)
    assert max(worst.values()) <= 5e-4, worst
    assert (num / den) ** 0.5 <= 1e-4


def test_training_heads_kernel_launches():
    """heads_epi 2 replaces the forward's head GEMM launches by one heads launch per forward: the
    guided main pass's two windows (pass 1's stratified points, then the guided ones) and the
    solar pass."""
    from spnerf_amd import _lib as L
    L.prof_reset()
    L.prof_enable(True)
    try:
        _render_train_heads({"heads_epi": 2}, True, 300, 64, True)
    finally:
        L.prof_enable(False)
    classes = L.prof_classes()
    assert "heads_train" in classes, classes
    assert L.prof_read("heads_train")["launches"] == 3   # main pass windows 0 and 1, solar pass


@pytest.mark.parametrize("sem,n,n_samples,guided", [(True, 300, 64, True), (False, 97, 40, False), (True, 97, 40, False),
                                                    (True, 1, 16, False)])
def test_heads_dx_chain_bitwise_equal(sem, n, n_samples, guided):
    """The heads' fused dX chain (k_heads_dx_bf16, option heads_dx 1: dS2, dZQ's sun half, dF and
    dZ_{L-1} in one launch, the main pass's every head and the solar pass's sun chain) equals the
    four layer-by-layer DMA GEMMs (heads_dx 0) bit for bit: the same MFMA sums in the same K order,
    the same epilogue arithmetic.  Sample counts that leave a partial 64-point tile included."""
    r0, g0 = _render_train_heads({"heads_dx": 0}, sem, n, n_samples, guided)
    r1, g1 = _render_train_heads({"heads_dx": 1}, sem, n, n_samples, guided)
    assert sorted(r0) == sorted(r1) and sorted(g0) == sorted(g1)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    for k in g0:
        assert torch.isfinite(g1[k]).all(), k
        assert torch.equal(g0[k], g1[k]), (k, (g0[k] - g1[k]).abs().max().item(), g0[k].abs().max().item())


def test_heads_dx_chain_launches():
    """One heads dX launch per saving forward's backward (the guided main pass's two windows share
    one backward; the solar pass has its own)."""
    from spnerf_amd import _lib as L
    L.prof_reset()
    L.prof_enable(True)
    try:
        _render_train_heads({"heads_dx": 1}, True, 300, 64, True)
    finally:
        L.prof_enable(False)
    assert L.prof_read("heads_dx")["launches"] == 2
