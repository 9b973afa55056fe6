"""C-ABI library: loads without a GPU, exports exactly what include/spnerf_amd.h declares,
agrees with the oracle on the parameter contract, and reports errors (no compute calls)."""
import ctypes
import os
import re

import pytest

import spnerf_amd
from spnerf_amd import _lib
from oracle.weights import ModelDims, param_specs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "spnerf_amd.h")).read()
    return sorted(set(re.findall(r"\b(spnerf_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_every_declared_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) == 39
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(_lib.SIGNATURES) == syms, "ctypes signature table out of sync with the header"
    assert L.spnerf_abi_version() == 2


def cfg_of(d: ModelDims):
    c = _lib.ModelCfg()
    c.width, c.layers, c.skip = d.width, d.layers, d.skips[0]
    c.n_freq = d.n_freq if d.mapping else 0
    c.sem_classes = d.num_sem_classes if d.sem else 0
    c.sem_dim = d.sem_dim
    c.beta, c.t_dim = int(d.beta), (d.t_dim if d.beta else 0)
    return c


@pytest.mark.parametrize("dims", [ModelDims(), ModelDims(width=64, sem=True), ModelDims(width=64, sem=True, beta=True),
                                  ModelDims(width=128, mapping=False), ModelDims(sem=True, num_sem_classes=5)])
def test_param_contract_matches_reference_order(dims):
    L = _lib.lib()
    c = cfg_of(dims)
    specs = param_specs(dims)
    assert L.spnerf_param_count(ctypes.byref(c)) == len(specs)
    buf = ctypes.create_string_buffer(128)
    for i, (name, shape, _) in enumerate(specs):
        r, k = ctypes.c_int64(), ctypes.c_int64()
        assert L.spnerf_param_info(ctypes.byref(c), i, buf, 128, ctypes.byref(r), ctypes.byref(k)) == 0
        got = (r.value, k.value) if k.value else (r.value,)
        assert buf.value.decode() == name and got == tuple(shape), (i, name)
    assert L.spnerf_packed_bytes(ctypes.byref(c)) > 4 * sum(int(__import__("numpy").prod(s)) for _, s, _ in specs)


def test_module_parameters_match_reference_state_dict():
    dims = ModelDims(sem=True, beta=True)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, beta=True, sem=True, t_embedding_dims=4)
    assert [(n, tuple(p.shape)) for n, p in m.named_parameters()] == [(n, tuple(s)) for n, s, _ in param_specs(dims)]
    assert m.number_of_outputs == dims.n_outputs
    assert [p.shape for p in m.canonical_parameters()] == [p.shape for p in m.parameters()]


def test_reference_default_param_count():
    m = spnerf_amd.SPNeRF(num_sem_classes=3, feat=512, mapping=True, sem=True)
    assert sum(p.numel() for p in m.parameters()) == 2_696_727


def test_errors_are_reported_not_fallen_back():
    L = _lib.lib()
    c = _lib.ModelCfg()
    c.width, c.layers, c.skip, c.n_freq = 100, 8, 4, 10      # width not a multiple of 64
    assert L.spnerf_param_count(ctypes.byref(c)) < 0
    assert b"width" in L.spnerf_last_error()
    assert L.spnerf_mlp_workspace_bytes(ctypes.byref(c), 10, 64, 0) == -1
    assert L.spnerf_sample_stratified(4, 64, None, 11, None, None, None, None) == -1
    assert b"NULL" in L.spnerf_last_error()


def test_product_path_refuses_cpu_tensors():
    import torch
    import types
    m = spnerf_amd.SPNeRF(feat=64, mapping=True)
    args = types.SimpleNamespace(n_samples=8, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                                 sc_lambda=0.0, margin=0, stdscale=1, chunk=5120, noise_std=0.0)
    with pytest.raises(_lib.SpnerfError, match="MI355X"):
        spnerf_amd.render_rays({"coarse": m}, args, torch.zeros(4, 11), None)
    with pytest.raises(ValueError):
        spnerf_amd.render_rays({"coarse": m}, types.SimpleNamespace(**{**vars(args), "model": "nerf"}), torch.zeros(4, 11), None)


def test_workspace_sizes_scale_with_points():
    L = _lib.lib()
    c = cfg_of(ModelDims(sem=True))
    a = L.spnerf_mlp_workspace_bytes(ctypes.byref(c), 1024, 64, _lib.SPNERF_MLP_SAVE)
    b = L.spnerf_mlp_workspace_bytes(ctypes.byref(c), 2048, 64, _lib.SPNERF_MLP_SAVE)
    n = L.spnerf_mlp_workspace_bytes(ctypes.byref(c), 1024, 64, 0)
    assert 0 < n < a < b


def test_seeded_init_matches_reference():
    """torch.manual_seed(7); SPNeRF(...) gives the reference's initial weights (fixture made by
    running the reference's constructor, tests/golden/gen_golden.py::init_weights)."""
    import numpy as np
    import torch
    import golden_util as gu
    with np.load(f"{gu.GOLDEN}/init_seed7.npz") as z:
        ref = {k: float(z[k]) for k in z.files}
    for tag, kw in (("w64_sem_beta", dict(num_sem_classes=3, feat=64, mapping=True, sem=True, beta=True,
                                          t_embedding_dims=4)),
                    ("w512", dict(feat=512, mapping=True))):
        torch.manual_seed(7)
        m = spnerf_amd.SPNeRF(**kw)
        Q = gu.param_projections([(n, tuple(p.shape)) for n, p in m.named_parameters()])
        for n, p in m.named_parameters():
            assert abs(p.detach().double().sum().item() - ref[f"{tag}|{n}|sum"]) <= 1e-9 * max(1.0, abs(ref[f"{tag}|{n}|sum"])), n
            proj = (p.detach().double() * torch.tensor(Q[n]).double()).sum().item()
            assert abs(proj - ref[f"{tag}|{n}|proj"]) <= 1e-9 * max(1.0, abs(ref[f"{tag}|{n}|proj"])), n


PRODUCT_OPTIONS = ("fused_trunk", "trunk_tile", "trunk_heads", "heads_epi", "trunk_l0", "pe_inline", "tn_group",
                   "tn_group_last", "defer_heads", "fused_bwd", "tn_bf16_variant", "tn_bf16_k64", "nt_f32_variant",
                   "pack_table", "prof_shapes")
ABLATION_OPTIONS = ("trunk_dbg", "trunk_var", "trunk_dreg", "trunk_bwd_dreg", "tn_bf16_pf", "tn_bf16_quad",
                    "tn_bf16_m16", "tn_bf16_rounds", "zsave", "trunk2", "trunk2_tile", "nt_bf16_ip", "tn_bf16_ip",
                    "emu_bf16", "bwd_streams", "heads_variant", "fused_heads", "tile_rowsum", "heads_dx")


def test_kernel_options_roundtrip_and_reject_unknown_names():
    L = _lib.lib()
    for name in PRODUCT_OPTIONS:
        old = _lib.get_option(name)
        _lib.set_option(name, old)
        assert _lib.get_option(name) == old
    assert _lib.get_option("fused_trunk") == 1 and _lib.get_option("nt_f32_variant") == 8
    assert L.spnerf_set_option(b"no_such_option", 1) < 0
    assert b"unknown option" in L.spnerf_last_error()
    with pytest.raises(_lib.SpnerfError):
        _lib.get_option("no_such_option")
    # profiling ablations that make the library compute invalid outputs exist only in a
    # -DSPN_ABLATIONS build, never in the product library
    for name in (b"trunk_dbg", b"trunk_var", b"heads_dbg"):
        assert L.spnerf_set_option(name, 1) < 0, name
    _lib.set_option("prof_shapes", 0)


def test_product_library_has_at_most_15_switches():
    """The product build accepts exactly its 15 documented kernel switches; the A/B switches of
    kernels measured slower (and the output-invalidating ablations) exist only in -DSPN_ABLATIONS
    builds — setting one raises OptionUnavailable (tests that need them skip)."""
    from spnerf_amd import _lib
    assert len(PRODUCT_OPTIONS) <= 15
    for n in PRODUCT_OPTIONS:
        assert _lib.has_option(n), n
        _lib.set_option(n, _lib.get_option(n))
    for n in ABLATION_OPTIONS:
        assert not _lib.has_option(n), n
        with pytest.raises(_lib.OptionUnavailable):
            _lib.set_option(n, 0)
