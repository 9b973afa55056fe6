"""Ray rendering — drop-in for ``modules/rendering.py`` of the reference.

Same functions, signatures, argument meaning, dictionary keys and error behaviour as the
reference; every step runs on the gfx950 kernels of libspnerf_amd.so:

==============================  ========================================  =====================
reference (rendering.py)         here                                      kernel
==============================  ========================================  =====================
stratified z  :131-144           ``stratified``                            k_stratified
inference pass 1 :157            σ-only MLP + weights-only composite       mlp + composite
                                 (training: the saving MLP's window 0)     mlp_forward_window
GenerateGuidedSamples :92-116    ``spnerf_sample_guided`` (+ sort, merge)  k_guided
  + sort / merge :165-167
inference pass 2 :169            full MLP + composite                      mlp + composite
                                 (training: the guided points only, the    mlp_forward_window,
                                 rows merged in sorted order)              k_merge_rows
fine pass :186-216               sample_pdf + sort + fine MLP/composite    k_sample_pdf, k_sort_rows
solar correction :171-177        σ+sun MLP + weights-only composite        mlp + composite
sample_pdf :14-55                ``sample_pdf``                            k_sample_pdf
sample_3sigma :58-73             ``sample_3sigma``                         k_sample_pdf (window)
==============================  ========================================  =====================
"""
from __future__ import annotations

import torch

from . import _lib
from .rng import begin_render, current_random_source, device_key
from .spnerf import (_result, composite, guided_inference_pass, guided_main_pass, inference_rays, mlp_saves,
                     pack_for_render)

# Training renders with guided sampling evaluate each main-pass point once (spnerf._GuidedMain):
# False = the reference's two evaluations of the stratified points (pass 1 σ-only, then the
# sorted union) — the A/B arm and the parity cross-check of tests/test_gpu_reuse.py
REUSE_PASS1 = True


def stratified(rays: torch.Tensor, n_samples: int, u: torch.Tensor = None, rng=None) -> torch.Tensor:
    """z = lower + (upper - lower)·u over [near, far] (rendering.py:131-144, perturb = 1); with
    ``rng`` (an spnerf_rng) instead of ``u`` the jitter is drawn on the device."""
    _lib.require_device(rays, u)
    rays = rays.contiguous().float()
    u = None if u is None else u.contiguous().float()
    z = torch.empty(rays.shape[0], n_samples, device=rays.device)
    _lib.check(_lib.lib().spnerf_sample_stratified(rays.shape[0], n_samples, _lib.ptr(rays), rays.stride(0), _lib.ptr(u),
                                                   _lib.ptr(z), _lib.rng_ref(rng), _lib.stream_of(rays)),
               "sample_stratified")
    return z


def sample_pdf(bins, weights, N_importance, det=False, eps=1e-5):
    """rendering.py:14-55.  (``det=True`` raises in the reference — 1-D ``u`` against a 2-D
    CDF in searchsorted — here it uses the intended ``linspace(0,1,N)`` for every ray.)"""
    _lib.require_device(bins, weights)
    B, nb = weights.shape
    key = keep = None
    if det:
        u = torch.linspace(0, 1, N_importance, device=bins.device).expand(B, N_importance).contiguous()
    else:
        key, keep = device_key(bins.device)
        u = None if key is not None else current_random_source().rand((B, N_importance), bins.device)
    out = torch.empty(B, N_importance, device=bins.device)
    b, w = bins.contiguous().float(), weights.contiguous().float()
    uu = None if u is None else u.contiguous().float()
    _lib.check(_lib.lib().spnerf_sample_pdf(B, nb, _lib.ptr(b), _lib.ptr(w), N_importance, _lib.ptr(uu), float(eps),
                                            _lib.ptr(out), _lib.rng_ref(key), _lib.stream_of(bins)), "sample_pdf")
    return out


def _bounds(near, far, device):
    nf = torch.stack([torch.as_tensor(near, dtype=torch.float32, device=device).reshape(()),
                      torch.as_tensor(far, dtype=torch.float32, device=device).reshape(())])
    return nf.contiguous()


def _window_samples(low, high, u, near, far):
    """Gaussian-binned window sampling at given uniforms u (B, N) (k_sample_pdf, window mode)."""
    B, N = u.shape
    lo = low.contiguous().float()          # converted tensors stay bound across the library call
    hi = high.contiguous().float()
    uu = u.contiguous().float()
    nf = _bounds(near, far, lo.device)
    out = torch.empty(B, N, device=lo.device)
    _lib.check(_lib.lib().spnerf_sample_3sigma(B, N, _lib.ptr(lo), _lib.ptr(hi), _lib.ptr(nf), _lib.ptr(uu), _lib.ptr(out),
                                               _lib.stream_of(lo)), "sample_3sigma")
    return out


def _uniforms(B, N, det, dev):
    if det:
        return torch.linspace(0, 1, N, device=dev).expand(B, N).contiguous()
    return current_random_source().rand((B, N), dev)


def sample_3sigma(low_3sigma, high_3sigma, N, det, near, far, device=None):
    """rendering.py:58-73: Gaussian-weighted bins over [low, high] clamped to [near, far]."""
    _lib.require_device(low_3sigma, high_3sigma)
    B = low_3sigma.shape[0]
    return _window_samples(low_3sigma, high_3sigma, _uniforms(B, N, det, low_3sigma.device), near, far)


def compute_samples_around_depth(res, N_samples, z_vals, perturb, near, far, device=None):
    """rendering.py:76-89."""
    depth, w = res["depth"], res["weights"]
    std = (((z_vals - depth.unsqueeze(-1)) ** 2) * w).sum(-1).sqrt()
    return sample_3sigma(depth - 3.0 * std, depth + 3.0 * std, N_samples, perturb == 0.0, near, far, device=device)


def _guided(res, z_vals, n, rays, mode, valid_depth, target_depths, target_std, clamp_nf=None):
    """Fused GenerateGuidedSamples + sort + merge.  Returns (z_sorted, z_unsort), both (B, 2n)."""
    B = z_vals.shape[0]
    dev = z_vals.device
    src = current_random_source()
    key, keep = device_key(dev, 2)   # on-device draws: slots key.slot (pred) and key.slot + 1 (GT)
    u_pred = None if key is not None else src.rand((B, n), dev).contiguous().float()   # rendering.py:35 via :87
    valid = tdep = tstd = u_gt = None
    td_stride = 2
    if mode == "train":
        assert valid_depth is not None, "valid_depth missing in training batch!"   # rendering.py:99
        valid = valid_depth.reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
        tdep = target_depths.to(device=dev, dtype=torch.float32).contiguous()
        td_stride = tdep.stride(0)
        tstd = target_std.reshape(-1).to(device=dev, dtype=torch.float32).contiguous()
        if key is None:
            u_gt = src.gt_uniform(valid, n, dev).contiguous().float()         # rendering.py:113
    z_sorted = torch.empty(B, 2 * n, device=dev)
    z_unsort = torch.empty(B, 2 * n, device=dev)
    if clamp_nf is None:
        clamp_nf = rays[0, 6:8]                                               # first ray: rendering.py:95,113
    depth, weights = res["depth"].contiguous(), res["weights"].contiguous()
    _lib.check(_lib.lib().spnerf_sample_guided(B, n, _lib.ptr(z_vals), _lib.ptr(depth),
                                               _lib.ptr(weights), _lib.ptr(clamp_nf), _lib.ptr(valid),
                                               _lib.ptr(tdep), td_stride, _lib.ptr(tstd), _lib.ptr(u_pred), _lib.ptr(u_gt),
                                               _lib.ptr(z_sorted), _lib.ptr(z_unsort), _lib.rng_ref(key),
                                               _lib.stream_of(z_vals)), "sample_guided")
    return z_sorted, z_unsort


def GenerateGuidedSamples(res, z_vals, N_samples, perturb, near, far, mode='test', valid_depth=None, target_depths=None,
                          target_std=None, device=None, margin=0, stdscale=1):
    """rendering.py:92-116 (``margin`` / ``stdscale`` are unused there too).  Samples come back
    in DRAW order, like the reference (render_rays sorts them afterwards, :165); the clamp bounds
    are near[0,0] / far[0,0] — the first ray of the chunk.  On rays with a depth prior (train)
    the window is the GT depth ± 3 target_std (:106-114).  render_rays itself uses the fused
    ``spnerf_sample_guided`` kernel, which also sorts and merges."""
    n0, f0 = near[0, 0], far[0, 0]
    z2 = compute_samples_around_depth(res, N_samples, z_vals, perturb, n0, f0, device=device)
    if mode == 'train':
        assert valid_depth is not None, 'valid_depth missing in training batch!'
        dev = z_vals.device
        valid = valid_depth.reshape(-1).to(device=dev, dtype=torch.int64)
        if perturb == 0.:
            u = _uniforms(valid.shape[0], N_samples, True, dev)
        else:   # one row of u per ray (rows of rays without a prior are unused)
            u = current_random_source().gt_uniform(valid, N_samples, dev)
        td = target_depths[:, 0].to(dev, torch.float32)
        ts = target_std.reshape(-1).to(dev, torch.float32)
        gt = _window_samples(td - 3. * ts, td + 3. * ts, u, n0, f0)
        z2 = torch.where((valid > 0).unsqueeze(-1), gt, z2)
    return z2


def _empty_batch(models, args, rays, ts, semantics, mode, valid_depth, target_depths, target_std, clamp_near_far):
    """An empty batch: the outputs of a one-ray placeholder render sliced to zero rows, so that they
    keep the reference's keys, trailing shapes and autograd connection (a backward through them
    leaves every parameter gradient zero).  The library's entry points take device pointers, which
    an empty tensor does not have; the placeholder ray (origin 0, direction -z, near 1, far 2, sun
    +z) keeps every value finite, so the zero gradients it receives stay zero."""
    one = torch.zeros(1, rays.shape[1], device=rays.device)
    one[0, 5], one[0, 6], one[0, 7] = -1.0, 1.0, 2.0
    if rays.shape[1] >= 11:
        one[0, 10] = 1.0

    def pick(t, fill):
        return None if t is None else torch.full((1,) + tuple(t.shape[1:]), fill, dtype=t.dtype, device=t.device)

    out = render_rays(models, args, one, pick(ts, 0), pick(semantics, 0), mode, pick(valid_depth, 0),
                      pick(target_depths, 1.5), pick(target_std, 0.1), clamp_near_far=clamp_near_far)
    return {k: v[:0] for k, v in out.items()}


def render_rays(models, args, rays, ts, semantics=None, mode='test', valid_depth=None, target_depths=None,
                target_std=None, *, clamp_near_far=None):
    """rendering.py:119-218 for the coarse SP-NeRF model; returns the same dictionary
    (keys suffixed ``_coarse``).  ``clamp_near_far`` (extension, device tensor of 2 floats)
    overrides the guided-sampling clamp bounds, which otherwise are the first ray's near/far
    like the reference — data-parallel ranks pass the GLOBAL batch's first ray."""
    N_samples = args.n_samples
    if args.model != "sp-nerf":
        raise ValueError(f'model {args.model} is not valid')
    _lib.require_device(rays)
    rays = rays.contiguous().float()
    B = rays.shape[0]
    if B == 0:
        return _empty_batch(models, args, rays, ts, semantics, mode, valid_depth, target_depths, target_std,
                            clamp_near_far)
    begin_render(rays.device)         # a keyed on-device random source starts a new step
    key, keep = device_key(rays.device)
    if key is not None:
        z_vals = stratified(rays, N_samples, rng=key)
    else:
        z_vals = stratified(rays, N_samples, current_random_source().rand((B, N_samples), rays.device))  # rendering.py:143
    model = models["coarse"]
    rays_t = None
    if args.beta:
        rays_t = models["t"](ts) if ts is not None else None                       # rendering.py:156
    sem = semantics if model.sem else None
    pk = pack_for_render(model)   # every pass of this render reads the same packed weights
    if args.guidedsample and REUSE_PASS1:
        # pass 1's rows ARE the main pass's rows at the stratified depths: each point is evaluated
        # once and the rows are composited in the sorted order (training: one saving forward in
        # two windows, spnerf._GuidedMain; no gradient: two forwards, guided_inference_pass)
        cnf = None if clamp_near_far is None else clamp_near_far.reshape(2).to(rays.device, torch.float32).contiguous()

        def guide(out1, z1):
            rgb1, depth1, w1, T1, sem1 = composite(model, out1, z1, args.noise_std, weights_only=True)
            return _guided({"depth": depth1, "weights": w1}, z1, N_samples, rays, mode, valid_depth, target_depths,
                           target_std, cnf)

        t_in = rays_t if model.beta else None
        run = guided_main_pass if mlp_saves(model, t_in) else guided_inference_pass
        out, z_vals, z_unsort = run(model, rays, z_vals, sem if model.sem else None, t_in, guide, pk)
        rgb, depth, w, T, sem_l = composite(model, out, z_vals, args.noise_std)
        result = _result(model, out, z_vals, rgb, depth, w, T, sem_l, z_unsort)
    elif args.guidedsample:
        with torch.no_grad():   # pass 1 feeds only the detached guided depths (rendering.py:164)
            res1 = inference_rays(model, args, rays, z_vals, 3, sem, rays_t, mode="sigma", pack=pk)
        cnf = None if clamp_near_far is None else clamp_near_far.reshape(2).to(rays.device, torch.float32).contiguous()
        z_vals, z_unsort = _guided(res1, z_vals, N_samples, rays, mode, valid_depth, target_depths, target_std, cnf)
        result = inference_rays(model, args, rays, z_vals, 3, sem, rays_t, z_vals_unsort=z_unsort, pack=pk)
    else:
        result = inference_rays(model, args, rays, z_vals, 3, sem, rays_t, pack=pk)
    if args.sc_lambda > 0:                                                           # rendering.py:171-177
        sc = inference_rays(model, args, rays, z_vals, 8, sem, rays_t, mode="sun", pack=pk)
        result["weights_sc"] = sc["weights"]
        result["transparency_sc"] = sc["transparency"]
        result["sun_sc"] = sc["sun"]
    out = {f"{k}_coarse": v for k, v in result.items()}
    if args.n_importance > 0:
        out = _fine(models, args, rays, ts, z_vals, out, semantics, rays_t)
    return out


def sort_rows(x: torch.Tensor) -> torch.Tensor:
    """torch.sort(x, -1)[0] for rows of ≤ 256 values (k_sort_rows)."""
    _lib.require_device(x)
    x = x.contiguous().float()
    out = torch.empty_like(x)
    _lib.check(_lib.lib().spnerf_sort_rows(x.shape[0], x.shape[1], _lib.ptr(x), _lib.ptr(out), _lib.stream_of(x)),
               "sort_rows")
    return out


def _fine(models, args, rays, ts, z_vals, result_, semantics, rays_t_coarse):
    """Hierarchical fine pass, rendering.py:186-216, reproduced as the reference returns it:
    with the solar pass on, ``result_`` is replaced by the fine solar inference's dictionary
    (:207), so the coarse keys are dropped and un-suffixed fine-solar keys appear."""
    n_imp = args.n_importance
    with torch.no_grad():
        mid = 0.5 * (z_vals[:, :-1] + z_vals[:, 1:])                               # :188
        z_ = sample_pdf(mid, result_["weights_coarse"][:, 1:-1], n_imp, det=False)  # :189 (perturb = 1)
        z_vals = sort_rows(torch.cat([z_vals, z_], -1))                             # :190
    model = models["fine"]
    rays_t = None
    if args.beta:
        rays_t = models['t'](ts) if ts else None                                    # :201, as written there
    sem = semantics if model.sem else None
    pk = pack_for_render(model)
    result = inference_rays(model, args, rays, z_vals, 3, sem, rays_t, pack=pk)
    if args.sc_lambda > 0:
        result_ = inference_rays(model, args, rays, z_vals, 8, sem, rays_t, pack=pk)  # :207 overwrites result_
        result["weights_sc"] = result_["weights"]
        result["transparency_sc"] = result_["transparency"]
        result["sun_sc"] = result_["sun"]
    for k in list(result.keys()):
        result_[f"{k}_fine"] = result[k]
    return result_
