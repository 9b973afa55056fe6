"""SP-NeRF model surface — drop-in for ``models/spnerf.py`` of the reference.

``SPNeRF`` keeps the reference's constructor signature, sub-module names and parameter
shapes (so reference checkpoints load with ``load_state_dict``, and ``torch.manual_seed(s)``
gives the same initial weights: the RNG-consuming constructors run in the reference's order,
spnerf.py:162-264), but its forward pass is the HIP library: positional encoding, the
8-layer SIREN trunk and every head run as gfx950 kernels (csrc/mlp.hip, csrc/gemm_f32.hip),
with a hand-written backward (``spnerf_mlp_backward``) behind ``torch.autograd.Function``.

``inference`` (spnerf.py:63-159) composites with the wavefront-scan kernels of
csrc/composite.hip.  Nothing here has a CPU path.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import (SPNERF_COMP_SUN_COLUMN, SPNERF_COMP_WEIGHTS_ONLY, SPNERF_MLP_ACCUMULATE, SPNERF_MLP_DEFER_TRUNK_WGRAD,
                   SPNERF_MLP_SAVE, SPNERF_MLP_SIGMA_ONLY, SPNERF_MLP_SUN_ONLY)
from .rng import current_random_source, device_key


class Mapping(torch.nn.Module):
    """Positional-encoding descriptor (spnerf.py:5-37): [sin(2^k x), cos(2^k x)], k < N_freqs.
    The encoding itself is computed inside the MLP kernels (k_encode); this module only
    carries the sizes the reference exposes."""

    def __init__(self, mapping_size, in_size, logscale=True):
        super().__init__()
        if not logscale:
            raise NotImplementedError("only log-scale frequency bands (the reference default) are supported")
        self.N_freqs = mapping_size
        self.in_channels = in_size
        self.out_channels = in_size * (2 * mapping_size + 1)
        self.freq_bands = 2 ** torch.linspace(0, mapping_size - 1, mapping_size)


class Siren(torch.nn.Module):
    """sin(w0 · x) activation marker (spnerf.py:40-46); fused into the GEMM epilogues."""

    def __init__(self, w0=1.0):
        super().__init__()
        self.w0 = w0

    def forward(self, x):  # kept for API completeness (elementwise, not on the render path)
        return torch.sin(self.w0 * x)


def sine_init(m):
    with torch.no_grad():
        if hasattr(m, "weight"):
            fan = m.weight.size(-1)
            m.weight.uniform_(-np.sqrt(6 / fan), np.sqrt(6 / fan))


def first_layer_sine_init(m):
    with torch.no_grad():
        if hasattr(m, "weight"):
            fan = m.weight.size(-1)
            m.weight.uniform_(-1 / fan, 1 / fan)


class SPNeRF(torch.nn.Module):
    """Same constructor and parameters as the reference SPNeRF (spnerf.py:162-271)."""

    def __init__(self, num_sem_classes=3, s_embedding_factor=1, layers=8, feat=256, mapping=False,
                 mapping_sizes=[10, 4], skips=[4], siren=True, t_embedding_dims=16, beta=False, sem=False,
                 precision="fp32"):
        super().__init__()
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        # MLP arithmetic (not a reference argument): "fp32" is the parity path; "bf16" keeps
        # activations and GEMM operands in bf16 with fp32 accumulation, fp32 layer 0, fp32
        # parameters and gradients — the counterpart of the reference's fp16 AMP training
        # (main.py:334-336, precision=16)
        self.precision = precision
        if not siren:
            raise NotImplementedError("the gfx950 trunk implements the SIREN activations (load_model never "
                                      "disables them, models/__init__.py:6-13)")
        if len(skips) > 1:
            raise NotImplementedError("one skip connection is supported (reference default skips=[4])")
        self.layers = layers
        self.skips = list(skips)
        self.t_embedding_dims = t_embedding_dims
        self.input_sizes = [3, 0]
        self.rgb_padding = 0.001
        self.beta = beta
        self.sem = sem
        self.num_sem_classes = num_sem_classes
        self.s_embedding_factor = s_embedding_factor
        self.semantic_size = num_sem_classes * s_embedding_factor if sem else 0
        self.feat = feat
        self.n_freq = mapping_sizes[0] if mapping else 0
        in_xyz = 2 * mapping_sizes[0] * 3 if mapping else 3
        self.mapping = [Mapping(ms, isz) for ms, isz in zip(mapping_sizes, self.input_sizes)] if mapping else \
            [torch.nn.Identity(), torch.nn.Identity()]
        H = feat // 2
        if sem:
            self.semantic_embedding = torch.nn.Embedding(num_sem_classes + 1, self.semantic_size,
                                                         padding_idx=num_sem_classes)
        self.input_size = in_xyz + self.semantic_size
        mods = []
        for i in range(layers):
            fan = self.input_size if i == 0 else (feat + self.input_size if i in self.skips else feat)
            mods += [torch.nn.Linear(fan, feat), Siren(30.0 if i == 0 else 1.0)]
        self.fc_net = torch.nn.Sequential(*mods)
        self.sigma_from_xyz = torch.nn.Sequential(torch.nn.Linear(feat, 1), torch.nn.Softplus())
        self.feats_from_xyz = torch.nn.Linear(feat, feat)
        if sem:
            self.logit_from_label = torch.nn.Sequential(torch.nn.Linear(feat, H), Siren(),
                                                        torch.nn.Linear(H, num_sem_classes))
        self.rgb_from_xyzdir = torch.nn.Sequential(torch.nn.Linear(feat, H), Siren(), torch.nn.Linear(H, 3),
                                                   torch.nn.Sigmoid())
        self.sun_v_net = torch.nn.Sequential(torch.nn.Linear(feat + 3, H), Siren(), torch.nn.Linear(H, H), Siren(),
                                             torch.nn.Linear(H, H), Siren(), torch.nn.Linear(H, 1), torch.nn.Sigmoid())
        self.sky_color = torch.nn.Sequential(torch.nn.Linear(3, H), torch.nn.ReLU(), torch.nn.Linear(H, 3),
                                             torch.nn.Sigmoid())
        self.fc_net.apply(sine_init)
        self.fc_net[0].apply(first_layer_sine_init)
        self.sun_v_net.apply(sine_init)
        self.sun_v_net[0].apply(first_layer_sine_init)
        if beta:
            self.beta_from_xyz = torch.nn.Sequential(torch.nn.Linear(t_embedding_dims + feat, H), Siren(),
                                                     torch.nn.Linear(H, 1), torch.nn.Softplus())
        self.number_of_outputs = 8 + (1 if beta else 0) + (num_sem_classes if sem else 0)
        self._cfg = None
        self._order = None
        self._packed = None
        self._pack_pool = []
        self._graph_packs = []   # packed-weight buffers captured into HIP graphs (kept alive)
        self._flat_grad = None
        self.flat_grads = False  # opt-in direct gradient path (use_flat_grads)
        # with flat gradients: one trunk weight-gradient GEMM per layer over all passes of a render
        self.defer_trunk_wgrad = True

    # ---------------------------------------------------------------- library plumbing
    def cfg(self) -> _lib.ModelCfg:
        if self._cfg is None:
            c = _lib.ModelCfg()
            c.width, c.layers = self.feat, self.layers
            c.skip = self.skips[0] if self.skips else -1
            c.n_freq = self.n_freq
            c.sem_classes = self.num_sem_classes if self.sem else 0
            c.sem_dim = self.semantic_size
            c.beta = 1 if self.beta else 0
            c.t_dim = self.t_embedding_dims if self.beta else 0
            c.dtype = 1 if self.precision == "bf16" else 0
            self._cfg = c
        return self._cfg

    def canonical_parameters(self):
        """Parameters in the library's canonical order (spnerf_param_info), shape-checked."""
        if self._order is None:
            L = _lib.lib()
            cfg = ctypes.byref(self.cfg())
            n = L.spnerf_param_count(cfg)
            if n < 0:
                _lib.check(n, "param_count")
            named = dict(self.named_parameters())
            order = []
            buf = ctypes.create_string_buffer(128)
            for i in range(n):
                r, c = ctypes.c_int64(), ctypes.c_int64()
                _lib.check(L.spnerf_param_info(cfg, i, buf, 128, ctypes.byref(r), ctypes.byref(c)), "param_info")
                name = buf.value.decode()
                shape = (r.value, c.value) if c.value else (r.value,)
                p = named[name]
                if tuple(p.shape) != shape:
                    raise _lib.SpnerfError(f"parameter {name}: module shape {tuple(p.shape)} != library {shape}")
                order.append(name)
            self._order = order
        named = dict(self.named_parameters())
        return [named[n] for n in self._order]

    def packed_weights(self, own: bool = False) -> torch.Tensor:
        """Kernel-layout copy of the weights, re-packed on every call (one ≈10 µs kernel).

        Change detection is not possible: ``torch.optim.Adam(fused=True)`` updates parameters
        in place without bumping ``_version``, so a version-keyed cache trains on stale weights.
        Re-packing unconditionally is also what a captured HIP graph of a training step needs
        (every replay re-packs the parameters the optimizer updated).

        ``own=True`` (a forward that saves for backward) packs into a buffer of its own, taken
        from a free list and handed back by ``release_packed`` after the backward: the backward
        then uses the weights of ITS forward even if the parameters change and another forward
        re-packs in between (autograd semantics).  Padding is zero from allocation and never
        written, so recycled buffers need no clearing."""
        params = self.canonical_parameters()
        _lib.require_device(params[0])
        dev = params[0].device
        if self._packed is not None and self._packed.device != dev:
            self._packed, self._pack_pool = None, []
        if own:
            buf = self._pack_pool.pop() if self._pack_pool else None
        else:
            buf = self._packed
        if buf is None:
            nbytes = _lib.lib().spnerf_packed_bytes(ctypes.byref(self.cfg()))
            buf = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
            if not own:
                self._packed = buf
        for p in params:
            if not p.is_contiguous() or p.dtype != torch.float32:
                raise _lib.SpnerfError("parameters must be contiguous float32")
        arr = (ctypes.c_void_p * len(params))(*[p.data_ptr() for p in params])
        _lib.check(_lib.lib().spnerf_pack_params(ctypes.byref(self.cfg()), arr, _lib.ptr(buf), _lib.stream_of(buf)),
                   "pack_params")
        return buf

    def release_graph_packs(self) -> list:
        """Hand over the packed-weight buffers captured into HIP graphs so far (see
        ``WeightPack.done``): the caller keeps them exactly as long as the graph(s) it captured
        (bench.TrainStep stores them beside its graph and drops both together).  Every replay writes
        the re-packed weights into these buffers, so they must outlive the graph: a buffer the
        capture took from the free list was allocated OUTSIDE the graph's private pool, and once
        unreferenced the caching allocator may hand it to eager tensors or, at the next
        ``torch.cuda.graph`` capture (whose ``__enter__`` calls ``torch.cuda.empty_cache()``),
        return its segment to the driver — a replay then writes unmapped memory (round 5's
        illegal-address fault)."""
        packs, self._graph_packs = self._graph_packs, []
        return packs

    def release_packed(self, buf: torch.Tensor) -> None:
        """Return a buffer from ``packed_weights(own=True)`` once its backward has run."""
        if buf is not None and buf is not self._packed and len(self._pack_pool) < 4:
            self._pack_pool.append(buf)

    def use_flat_grads(self, on: bool = True) -> "SPNeRF":
        """Opt in to the direct gradient path (the training loop's ``loss.backward()`` into
        leaf ``.grad``s, as bench.py and dp do): the MLP backward then adds every parameter's
        gradient straight into one flat buffer whose views ARE the ``.grad``s (no per-parameter
        autograd accumulation, no flatten for the all-reduce), bypassing autograd's gradient
        return — so per-parameter hooks do not fire and ``torch.autograd.grad`` must not be
        used on the parameters.  Off by default: gradients go back through autograd."""
        self.flat_grads = bool(on)
        return self

    def flat_grad_target(self, params):
        """Where the MLP backward accumulates parameter gradients directly: with
        ``use_flat_grads`` on and EVERY canonical parameter requiring grad, the model's flat
        gradient buffer, when every parameter's ``.grad`` is its view — or, when every
        ``.grad`` is None, the buffer zeroed, with its views installed as the ``.grad``s.  None
        otherwise (the gradients then go back through autograd; a frozen parameter never gets
        a ``.grad`` here)."""
        if not self.flat_grads or not all(p.requires_grad for p in params):
            return None
        fb = self._flat_grad
        if all(p.grad is None for p in params):
            total = sum(p.numel() for p in params)
            dev = params[0].device
            if fb is None or fb.numel() != total or fb.device != dev:
                fb = torch.empty(total, dtype=torch.float32, device=dev)
                self._flat_grad = fb
            fb.zero_()
            off = 0
            for p in params:
                p.grad = fb[off:off + p.numel()].view_as(p)
                off += p.numel()
            return fb
        if fb is None:
            return None
        base, off = fb.data_ptr(), 0
        for p in params:
            g = p.grad
            if g is None or g.data_ptr() != base + 4 * off or g.shape != p.shape or not g.is_contiguous():
                return None
            off += p.numel()
        return fb

    def invalidate_packed(self) -> None:
        """Kept for callers that prepared a graph capture with it: packing is unconditional."""

    def set_precision(self, precision: str) -> "SPNeRF":
        """Switch the MLP arithmetic ("fp32" | "bf16"); parameters are unchanged."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self.precision = precision
        self._cfg, self._packed, self._pack_pool = None, None, []
        return self

    def _apply(self, fn, *args, **kwargs):
        self._packed, self._pack_pool = None, []
        return super()._apply(fn, *args, **kwargs)

    # ---------------------------------------------------------------- reference forward API
    def forward(self, input_xyz, input_dir=None, input_sun_dir=None, input_t=None, input_s=None, sigma_only=False):
        """Per-point network (spnerf.py:273-369) on the HIP kernels: (P,3) → (P, number_of_outputs)
        with columns [rgb3, σ, sun, sky3, (β), sem] (or σ (P,1) if ``sigma_only``)."""
        _lib.require_device(input_xyz)
        P = input_xyz.shape[0]
        sun = input_sun_dir if input_sun_dir is not None else torch.zeros_like(input_xyz)
        pts = torch.cat([input_xyz.float(), torch.zeros(P, 5, device=input_xyz.device), sun.float()], 1)
        z = torch.zeros(P, 1, device=input_xyz.device)
        labels = None
        if self.sem:
            if input_s is None:
                raise ValueError("semantic SPNeRF needs input_s")
            labels = input_s.reshape(-1).long()
        t = input_t.float() if self.beta else None
        out = run_mlp(self, pts, z, 3, labels, t, sigma_only=sigma_only)
        return out[:, 3:4] if sigma_only else out


# ------------------------------------------------------------------------------------------
# autograd functions
# ------------------------------------------------------------------------------------------

class WeightPack:
    """One packed copy of a model's weights shared by the MLP calls of one render (all passes
    of a render_rays call see the same parameters).  A buffer of its own (``owned``) goes back to
    the model's free list once the last backward that reads it has run."""

    def __init__(self, model, owned: bool):
        self.model, self.owned, self.pending = model, owned, 0
        self.nsave = 0          # saving forwards of this render (main pass, solar pass, ...)
        self.deferred = []      # backwards that left their trunk weight gradients (see _MLP.backward)
        self.buf = model.packed_weights(own=owned)

    def flush_trunk_wgrad(self):
        """The trunk layers' weight gradients of the deferred backwards: ONE weight-gradient GEMM
        per layer over their points (spnerf_mlp_trunk_wgrad), added into the model's flat
        gradient.  Queued as an autograd-engine callback, so it runs once the whole backward pass
        is done, whichever of the render's passes were differentiated."""
        if not self.deferred:
            return
        segs, self.deferred = self.deferred, []
        grad, stream = segs[0][4], segs[0][5]
        n = len(segs)
        wss = (ctypes.c_void_p * n)(*[t[0].data_ptr() for t in segs])
        nr = (ctypes.c_int64 * n)(*[t[1] for t in segs])
        ns = (ctypes.c_int32 * n)(*[t[2] for t in segs])
        fl = (ctypes.c_int32 * n)(*[t[3] for t in segs])
        # on the stream the backwards ran on (an engine callback may run on another thread / stream)
        _lib.check(_lib.lib().spnerf_mlp_trunk_wgrad(ctypes.byref(self.model.cfg()), n, wss, nr, ns, fl, _lib.ptr(grad),
                                                      ctypes.c_void_p(stream.cuda_stream)), "mlp_trunk_wgrad")

    def done(self):
        self.pending -= 1
        if self.pending == 0 and self.owned:
            # a buffer captured into a HIP graph is re-packed by every replay: it never returns
            # to the free list, where a later eager forward could take it while a replay's
            # backward still reads it
            if not torch.cuda.is_current_stream_capturing():
                self.model.release_packed(self.buf)
            else:
                # ... and it must stay ALLOCATED for the graph's lifetime: a buffer taken from the
                # free list was allocated outside the capture, so with its last reference gone
                # the caching allocator would hand its memory to later eager tensors, or release
                # it to the driver at the next capture's empty_cache(), while every replay still
                # writes the packed weights into it (SPNeRF.release_graph_packs)
                self.model._graph_packs.append(self.buf)
            self.buf = None


def pack_for_render(model) -> "WeightPack":
    """Pack once for a whole render: own buffer when gradients may be taken."""
    return WeightPack(model, owned=torch.is_grad_enabled())


class _MLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, pack, rays, dir_offset, z, labels, temb, flags, *params):
        cfg = model.cfg()
        B, S = z.shape
        dev = rays.device
        need_grad = bool(flags & SPNERF_MLP_SAVE)
        L = _lib.lib()
        wsb = L.spnerf_mlp_workspace_bytes(ctypes.byref(cfg), B, S, flags)
        if wsb < 0:
            _lib.check(-1, "workspace_bytes")
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        out = torch.empty(B * S, model.number_of_outputs, dtype=torch.float32, device=dev)
        if pack is None or (need_grad and not pack.owned):
            pack = WeightPack(model, owned=need_grad)
        packed = pack.buf
        _lib.check(L.spnerf_mlp_forward(ctypes.byref(cfg), _lib.ptr(packed), _lib.ptr(rays), rays.stride(0), dir_offset,
                                        B, S, _lib.ptr(z), _lib.ptr(labels), _lib.ptr(temb), flags, _lib.ptr(ws),
                                        _lib.ptr(out), _lib.stream_of(rays)), "mlp_forward")
        if need_grad:
            pack.pending += 1
            pack.nsave += 1
            ctx.model, ctx.flags, ctx.ws, ctx.pack, ctx.packed = model, flags, ws, pack, packed
            ctx.shape = (B, S)
            ctx.save_for_backward(rays, labels, temb)
        return out

    @staticmethod
    def backward(ctx, d_out):
        rays, labels, temb = ctx.saved_tensors
        if ctx.ws is None:
            raise RuntimeError("SPNeRF MLP backward called twice on the same forward (its activations are freed)")
        B, S = ctx.shape
        gt, grads = _mlp_backward(ctx.model, ctx.pack, ctx.packed, ctx.ws, ctx.flags, rays, labels, temb, B, S,
                                  d_out.contiguous(), temb is not None and ctx.needs_input_grad[6])
        ctx.pack = ctx.packed = None
        ctx.ws = None
        return (None, None, None, None, None, None, gt, None, *grads)


def _mlp_backward(model, pack, packed, ws, fwd_flags, rays, labels, temb, B, S, d_out, temb_grad):
    """spnerf_mlp_backward of one saving forward's workspace: the parameter gradients straight into
    the model's flat gradient (``use_flat_grads``) or returned per parameter, and the t-embedding's.
    Returns (grad_t_emb or None, per-parameter gradients or Nones)."""
    params = model.canonical_parameters()
    gt = torch.empty_like(temb) if temb_grad else None
    flags = fwd_flags
    grad = model.flat_grad_target(params)
    direct = grad is not None
    # A render with several saving passes (main + solar correction) over one bf16 trunk: each
    # backward leaves the trunk's weight gradients, and one GEMM per layer over all the passes'
    # points runs when the backward pass ends (half the launches and split reductions)
    defer = (direct and pack.nsave > 1 and model.precision == "bf16" and model.defer_trunk_wgrad
             and _lib.lib().spnerf_mlp_trunk_wgrad(ctypes.byref(model.cfg()), 0, None, None, None, None, None,
                                                   None) == 1)
    if direct:   # add straight into the .grad views (the library's fixed-order reductions)
        flags |= SPNERF_MLP_ACCUMULATE
    else:
        grad = torch.empty(sum(p.numel() for p in params), dtype=torch.float32, device=rays.device)
    if defer:
        flags |= SPNERF_MLP_DEFER_TRUNK_WGRAD
    _lib.check(_lib.lib().spnerf_mlp_backward(ctypes.byref(model.cfg()), _lib.ptr(packed), _lib.ptr(rays),
                                              rays.stride(0), B, S, _lib.ptr(labels), _lib.ptr(temb), flags,
                                              _lib.ptr(ws), _lib.ptr(d_out), _lib.ptr(grad),
                                              _lib.ptr(gt), _lib.stream_of(rays)), "mlp_backward")
    if defer:
        if not pack.deferred:
            torch.autograd.Variable._execution_engine.queue_callback(pack.flush_trunk_wgrad)
        pack.deferred.append((ws, B, S, fwd_flags, grad, torch.cuda.current_stream(rays.device)))
    pack.done()
    if direct:
        return gt, [None] * len(params)
    grads, off = [], 0
    for p in params:
        grads.append(grad[off:off + p.numel()].view_as(p))
        off += p.numel()
    return gt, grads


class _GuidedMain(torch.autograd.Function):
    """render_rays' guided main pass (rendering.py:157-170) with every point evaluated ONCE.

    The reference runs the MLP over the 64 stratified depths (pass 1: its depth and weights place
    the guided samples) and then again over the sorted union of those depths and the 64 guided
    ones; the union's stratified points are pass 1's points (the same o + d·z, :147 / :168), so
    their MLP rows are the same.  Here pass 1 is the first window of ONE saving forward
    (``spnerf_mlp_forward_window``: rays [0, B) of a (2B rays, S) workspace), ``guide`` composites
    its σ (weights only, no gradient, :157 feeds only the detached guided depths) and draws the
    guided depths, the guided points are the second window (rays [B, 2B)), and
    ``spnerf_merge_samples`` gathers both windows' rows into the sorted order the composite reads.
    The backward scatters the sorted rows' gradients back (``spnerf_merge_samples_backward``) and
    runs ONE MLP backward over the 2B "rays" (the rays / labels / t-embeddings repeated).  Draws
    happen in the reference's order: pass 1's σ noise, the guided windows, then the caller's."""

    @staticmethod
    def forward(ctx, model, pack, rays, z1, labels, temb, guide, *params):
        cfg = model.cfg()
        B, S = z1.shape
        dev = rays.device
        NO = model.number_of_outputs
        flags = SPNERF_MLP_SAVE
        L = _lib.lib()
        wsb = L.spnerf_mlp_workspace_bytes(ctypes.byref(cfg), 2 * B, S, flags)
        if wsb < 0:
            _lib.check(-1, "workspace_bytes")
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        seg = torch.empty(2 * B * S, NO, dtype=torch.float32, device=dev)
        packed = pack.buf

        def window(r0, z):
            _lib.check(L.spnerf_mlp_forward_window(ctypes.byref(cfg), _lib.ptr(packed), _lib.ptr(rays), rays.stride(0), 3,
                                                   2 * B, r0, B, S, _lib.ptr(z), z.stride(0), _lib.ptr(labels),
                                                   _lib.ptr(temb), flags, _lib.ptr(ws), _lib.ptr(seg[r0 * S:(r0 + B) * S]),
                                                   _lib.stream_of(rays)), "mlp_forward_window")

        window(0, z1)
        z_sorted, z_unsort = guide(seg[:B * S], z1)
        window(B, z_unsort[:, S:])   # the sorted guided depths, read in place (row stride 2S)
        out = torch.empty(B * 2 * S, NO, dtype=torch.float32, device=dev)
        _lib.check(L.spnerf_merge_samples(B, S, S, _lib.ptr(z_unsort), _lib.ptr(seg), _lib.ptr(seg[B * S:]), NO,
                                          _lib.ptr(out), _lib.stream_of(rays)), "merge_samples")
        pack.pending += 1
        pack.nsave += 1
        ctx.model, ctx.ws, ctx.pack, ctx.packed, ctx.B, ctx.S = model, ws, pack, packed, B, S
        ctx.rays2 = torch.cat([rays, rays])
        ctx.labels2 = None if labels is None else torch.cat([labels, labels])
        ctx.temb2 = None if temb is None else torch.cat([temb, temb])
        ctx.z_unsort = z_unsort
        ctx.mark_non_differentiable(z_sorted, z_unsort)
        ctx.set_materialize_grads(False)   # the depth outputs take no gradient: no zero fills for them
        return out, z_sorted, z_unsort

    @staticmethod
    def backward(ctx, d_out, _dzs, _dzu):
        if ctx.ws is None:
            raise RuntimeError("SPNeRF MLP backward called twice on the same forward (its activations are freed)")
        B, S, NO = ctx.B, ctx.S, ctx.model.number_of_outputs
        if d_out is None:   # the rows took no gradient (the backward still consumes the workspace)
            d_out = torch.zeros(B * 2 * S, NO, dtype=torch.float32, device=ctx.rays2.device)
        d_out = d_out.contiguous()
        d_seg = torch.empty(2 * B * S, NO, dtype=torch.float32, device=d_out.device)
        _lib.check(_lib.lib().spnerf_merge_samples_backward(B, S, S, _lib.ptr(ctx.z_unsort), _lib.ptr(d_out), NO,
                                                            _lib.ptr(d_seg), _lib.ptr(d_seg[B * S:]), _lib.stream_of(d_out)),
                   "merge_samples_backward")
        temb_grad = ctx.temb2 is not None and ctx.needs_input_grad[5]
        gt2, grads = _mlp_backward(ctx.model, ctx.pack, ctx.packed, ctx.ws, SPNERF_MLP_SAVE, ctx.rays2, ctx.labels2,
                                   ctx.temb2, 2 * B, S, d_seg, temb_grad)
        ctx.pack = ctx.packed = ctx.ws = None
        gt = None if gt2 is None else gt2[:B] + gt2[B:]
        return (None, None, None, None, None, gt, None, *grads)


def mlp_saves(model: SPNeRF, temb=None) -> bool:
    """Whether run_mlp would run a saving (differentiable) forward."""
    return torch.is_grad_enabled() and (any(p.requires_grad for p in model.canonical_parameters()) or
                                        (temb is not None and temb.requires_grad))


def guided_inference_pass(model: SPNeRF, rays, z1, labels, temb, guide, pack: "WeightPack"):
    """The no-gradient twin of ``guided_main_pass``: pass 1 runs every head over the stratified
    depths (instead of σ alone), the second forward only the guided ones, and
    ``spnerf_merge_samples`` gathers both into the sorted order — each point evaluated once."""
    B, S = z1.shape
    with torch.no_grad():
        out1 = run_mlp(model, rays, z1, 3, labels, temb, pack=pack)
        z_sorted, z_unsort = guide(out1, z1)
        out2 = run_mlp(model, rays, z_unsort[:, S:].contiguous(), 3, labels, temb, pack=pack)
        out = torch.empty(B * 2 * S, model.number_of_outputs, dtype=torch.float32, device=rays.device)
        _lib.check(_lib.lib().spnerf_merge_samples(B, S, S, _lib.ptr(z_unsort), _lib.ptr(out1), _lib.ptr(out2),
                                                   model.number_of_outputs, _lib.ptr(out), _lib.stream_of(out1)),
                   "merge_samples")
    return out, z_sorted, z_unsort


def guided_main_pass(model: SPNeRF, rays, z1, labels, temb, guide, pack: "WeightPack"):
    """The guided main pass's MLP rows in sorted depth order (see _GuidedMain): returns (out,
    z_sorted, z_unsort) with out (B·2S, number_of_outputs)."""
    _lib.require_device(rays, z1, labels, temb)
    rays = rays.contiguous().float()
    z1 = z1.contiguous().float()
    if labels is not None:
        labels = labels.reshape(-1).to(torch.int64).contiguous()
    if temb is not None:
        temb = temb.contiguous().float()
    if not pack.owned:
        raise _lib.SpnerfError("guided_main_pass needs a render pack of its own (pack_for_render under grad)")
    return _GuidedMain.apply(model, pack, rays, z1, labels, temb, guide, *model.canonical_parameters())


def run_mlp(model: SPNeRF, rays: torch.Tensor, z: torch.Tensor, dir_offset: int, labels=None, temb=None,
            sigma_only=False, sun_only=False, pack: Optional[WeightPack] = None) -> torch.Tensor:
    """out (B·S, number_of_outputs) for xyz = rays[:, 0:3] + rays[:, dir:dir+3] · z."""
    _lib.require_device(rays, z, labels, temb)
    rays = rays.contiguous().float()
    z = z.contiguous().float()
    if labels is not None:
        labels = labels.reshape(-1).to(torch.int64).contiguous()
    if temb is not None:
        temb = temb.contiguous().float()
    flags = (SPNERF_MLP_SIGMA_ONLY if sigma_only else 0) | (SPNERF_MLP_SUN_ONLY if sun_only else 0)
    params = model.canonical_parameters()
    if torch.is_grad_enabled() and (any(p.requires_grad for p in params) or (temb is not None and temb.requires_grad)):
        if sigma_only:
            raise _lib.SpnerfError("sigma-only passes are not differentiable (run them under torch.no_grad())")
        flags |= SPNERF_MLP_SAVE
        return _MLP.apply(model, pack, rays, dir_offset, z, labels, temb, flags, *params)
    # No autograd: ray chunks of at most max_points_per_call() points each write a slice of one
    # output (the reference's args.chunk loop, spnerf.py:98, with chunks sized by the library's
    # per-call limit instead of 5120 points).
    B, S = z.shape
    cb = max(1, max_points_per_call(model) // S)
    if pack is None:
        pack = WeightPack(model, owned=False)
    if B <= cb:
        return _MLP.apply(model, pack, rays, dir_offset, z, labels, temb, flags, *params)
    out = torch.empty(B * S, model.number_of_outputs, dtype=torch.float32, device=rays.device)
    for i0 in range(0, B, cb):
        i1 = min(B, i0 + cb)
        out[i0 * S:i1 * S] = _MLP.apply(model, pack, rays[i0:i1], dir_offset, z[i0:i1],
                                        None if labels is None else labels[i0:i1],
                                        None if temb is None else temb[i0:i1], flags, *params)
    return out


def max_points_per_call(model: SPNeRF) -> int:
    """Largest B·S one spnerf_mlp_forward accepts (mlp.hip: P < 2^31 / max(NQ, NG))."""
    H = model.feat // 2
    nq = 2 * H + (H if model.beta else 0)
    ng = model.feat + (H if model.sem else 0)
    return ((1 << 31) - 1) // max(nq, ng)


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, z, noise, noise_std, sem_col, n_sem, weights_only, rng=None, rng_keep=None, sun_col=False):
        B, S = z.shape
        NO = out.shape[1]
        dev = out.device
        f = SPNERF_COMP_WEIGHTS_ONLY if weights_only else 0
        if weights_only and sun_col:   # the first output is then the sun column (B, S) of out
            f |= SPNERF_COMP_SUN_COLUMN
            rgb = torch.empty(B, S, device=dev)
        else:
            rgb = torch.empty(B, 3, device=dev) if not weights_only else torch.empty(0, device=dev)
        sem = torch.empty(B, n_sem, device=dev) if (n_sem and not weights_only) else torch.empty(0, device=dev)
        depth = torch.empty(B, device=dev)
        w = torch.empty(B, S, device=dev)
        T = torch.empty(B, S, device=dev)
        _lib.check(_lib.lib().spnerf_composite_forward(B, S, _lib.ptr(z), _lib.ptr(out), NO, _lib.ptr(noise),
                                                       float(noise_std), sem_col, n_sem, f, _lib.ptr(rgb), _lib.ptr(depth),
                                                       _lib.ptr(w), _lib.ptr(T), _lib.ptr(sem), _lib.rng_ref(rng),
                                                       _lib.stream_of(out)), "composite_forward")
        ctx.save_for_backward(out, z, noise)
        ctx.cfg = (float(noise_std), sem_col, n_sem, f)
        ctx.rng, ctx.rng_keep = rng, rng_keep   # the backward redraws the same on-device noise
        ctx.set_materialize_grads(False)
        return rgb, depth, w, T, sem

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_w, g_T, g_sem):
        out, z, noise = ctx.saved_tensors
        noise_std, sem_col, n_sem, f = ctx.cfg
        B, S = z.shape
        # contiguous copies stay bound to names until the library call has been issued
        g_rgb, g_depth, g_w, g_T, g_sem = (None if g is None else g.contiguous() for g in (g_rgb, g_depth, g_w, g_T, g_sem))
        d_out = torch.empty_like(out)
        _lib.check(_lib.lib().spnerf_composite_backward(B, S, _lib.ptr(z), _lib.ptr(out), out.shape[1], _lib.ptr(noise),
                                                        noise_std, sem_col, n_sem, f, _lib.ptr(g_rgb),
                                                        _lib.ptr(g_depth), _lib.ptr(g_w), _lib.ptr(g_T),
                                                        _lib.ptr(g_sem), _lib.ptr(d_out), _lib.rng_ref(ctx.rng),
                                                        _lib.stream_of(out)), "composite_backward")
        return d_out, None, None, None, None, None, None, None, None, None


def composite(model: SPNeRF, out: torch.Tensor, z: torch.Tensor, noise_std: float, weights_only=False, sun_col=False):
    """inference()'s compositing (spnerf.py:109-157).  ``sun_col`` (weights-only passes): the
    first output is the sun-visibility column of ``out`` (B, S), whose gradient the composite
    backward writes into d_out's sun column (the solar pass's sun_sc, rendering.py:177)."""
    B, S = z.shape
    key, keep = device_key(z.device)   # on-device σ noise: a slot per inference call, drawn or not
    noise = None if key is not None else current_random_source().noise((B, S), z.device, noise_std)   # spnerf.py:122
    if noise is not None:
        noise = noise.contiguous().float()
    sem_col = 8 + (1 if model.beta else 0)
    n_sem = model.num_sem_classes if model.sem else 0
    return _Composite.apply(out, z.contiguous(), noise, noise_std, sem_col, n_sem, weights_only,
                            key if noise_std != 0 else None, keep, sun_col)


def _result(model, out, z, rgb, depth, w, T, sem, z_unsort=None, sun=None):
    B, S = z.shape
    o = out.view(B, S, model.number_of_outputs)
    res = {"rgb": rgb, "depth": depth, "weights": w, "transparency": T, "albedo": o[..., :3],
           "sun": o[..., 4:5] if sun is None else sun.view(B, S, 1), "sky": o[..., 5:8], "z_vals": z}
    if z_unsort is not None:
        res["z_vals_unsort"] = z_unsort
    col = 8
    if model.beta:
        res["beta"] = o[..., col:col + 1]
        col += 1
    if model.sem:
        res["sem_logits"] = sem
    return res


def inference_rays(model: SPNeRF, args, rays, z_vals, dir_offset=3, semantics=None, rays_t=None, z_vals_unsort=None,
                   mode="full", pack: Optional[WeightPack] = None):
    """inference() over rays given by (origin, direction) + depths, without materialising xyz:
    mode 'full' (all heads), 'sun' (σ + sun, the solar-correction pass) or 'sigma'.  ``pack``:
    the weights packed once for a whole render (``pack_for_render``)."""
    out = run_mlp(model, rays, z_vals, dir_offset, semantics if model.sem else None, rays_t if model.beta else None,
                  sigma_only=mode == "sigma", sun_only=mode == "sun", pack=pack)
    if mode == "sun":   # the solar pass: sun_sc straight from the composite (its gradient fused there)
        sun, depth, w, T, sem = composite(model, out, z_vals, args.noise_std, weights_only=True, sun_col=True)
        return _result(model, out, z_vals, torch.empty(0, device=out.device), depth, w, T, sem, z_vals_unsort, sun=sun)
    rgb, depth, w, T, sem = composite(model, out, z_vals, args.noise_std, weights_only=mode != "full")
    return _result(model, out, z_vals, rgb, depth, w, T, sem, z_vals_unsort)


def inference(model, args, rays_xyz, z_vals, rays_d=None, sun_d=None, rays_t=None, semantics=None, z_vals_unsort=None):
    """Drop-in for spnerf.py:63 on explicit sample positions rays_xyz (N_rays, N_samples, 3)."""
    _lib.require_device(rays_xyz, z_vals)
    B, S = z_vals.shape
    pts = rays_xyz.reshape(B * S, 3).float()
    sd = torch.zeros(B, 3, device=pts.device) if sun_d is None else sun_d.float()
    rays = torch.cat([pts, torch.zeros(B * S, 5, device=pts.device), sd.repeat_interleave(S, 0)], 1)
    lab = semantics.reshape(-1).repeat_interleave(S, 0) if (semantics is not None and model.sem) else None
    t = rays_t.repeat_interleave(S, 0) if (rays_t is not None and model.beta) else None
    out = run_mlp(model, rays, torch.zeros(B * S, 1, device=pts.device), 3, lab, t)
    rgb, depth, w, T, sem = composite(model, out, z_vals.contiguous().float(), args.noise_std)
    return _result(model, out, z_vals, rgb, depth, w, T, sem, z_vals_unsort)
