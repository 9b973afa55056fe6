"""Random source of the render path.

The reference draws every random tensor from torch's global generator, in a fixed order
(SURVEY.md §4): stratified jitter ``rand (B,S)`` (rendering.py:143), σ noise ``randn``
per inference call (spnerf.py:122), ``rand (B,S)`` for the predicted-depth window
(rendering.py:35 via :87) and ``rand (B_valid,S)`` for the GT window (:113).

``TorchRandom`` (the default) draws the same tensors with torch on the rays' device; it
skips the σ-noise draw when ``noise_std == 0`` (the product with 0 is exactly 0) and draws
the GT-window ``u`` for every ray, indexed by ray, so no host synchronisation is needed to
count the valid rays.  ``ReplayRandom`` hands back pre-recorded draws (the reference's, in
the parity tests) in the reference's order and shapes.  ``PhiloxRandom`` draws nothing on the
host: the kernels that consume a draw generate it themselves (counter-based Philox4x32-10,
spnerf_rng in include/spnerf_amd.h) from (seed, step, global ray id, draw slot), so the draws
of a ray do not depend on which rank renders it or with which other rays, and a render launches
no RNG kernels.
"""
from __future__ import annotations

import contextlib
import threading

import torch


class TorchRandom:
    def rand(self, shape, device):
        return torch.rand(shape, device=device)

    def noise(self, shape, device, noise_std):
        if noise_std == 0:
            return None
        return torch.randn(shape, device=device)

    def gt_uniform(self, valid_mask, n, device):
        return torch.rand((valid_mask.shape[0], n), device=device)


class ReplayRandom:
    """Replays a list of (kind, array) draws recorded from the reference."""

    def __init__(self, draws):
        self.draws = list(draws)
        self.used = 0

    def _next(self, kind, shape):
        k, arr = self.draws[self.used]
        if k != kind or tuple(arr.shape) != tuple(shape):
            raise AssertionError(f"draw {self.used}: expected {kind}{tuple(shape)}, recorded {k}{tuple(arr.shape)}")
        self.used += 1
        return arr

    def rand(self, shape, device):
        return torch.as_tensor(self._next("rand", shape), device=device)

    def noise(self, shape, device, noise_std):
        return torch.as_tensor(self._next("randn", shape), device=device)

    def gt_uniform(self, valid_mask, n, device):
        sel = (valid_mask.reshape(-1) > 0).cpu()
        arr = torch.as_tensor(self._next("rand", (int(sel.sum()), n)))
        full = torch.zeros(valid_mask.shape[0], n)
        full[sel] = arr
        return full.to(device)


class PhiloxRandom:
    """On-device draws keyed by (seed, step, global ray id, slot) — SURVEY §8(b).

    Each ``render_rays`` is one step: ``begin_render`` advances the step in a device counter
    (an in-place add, so a captured HIP graph advances it on every replay) and snapshots
    {seed, step} into a tensor of its own that the render's kernels — and its backward's — read.
    Within a render every draw stream takes the next slot, in the render's fixed call order (the
    guided sampler takes two).  ``ray_offset`` is the global id of the call's first ray: a
    data-parallel rank passes rank · rays_per_rank and draws what a single process rendering
    the whole batch draws for those rays."""

    on_device = True

    def __init__(self, seed: int = 0, ray_offset: int = 0):
        self.seed, self.ray_offset = int(seed), int(ray_offset)
        self._state = None
        self._snap = None
        self._slot = 0
        self._host_step = -1   # host mirror of the device step (eager renders only; see _gen)

    def begin_render(self, device):
        if self._state is None:
            self._state = torch.tensor([self.seed, self._host_step], dtype=torch.int64, device=device)
        elif self._state.device != torch.device(device):
            # moved with its DEVICE step: graph replays advance that one, not the host mirror
            self._state = self._state.to(device)
        # state[1] += 1 and the snapshot in one launch (spnerf_rng_begin)
        from . import _lib
        self._snap = torch.empty(2, dtype=torch.int64, device=self._state.device)
        _lib.check(_lib.lib().spnerf_rng_begin(_lib.ptr(self._state), _lib.ptr(self._snap), _lib.stream_of(self._state)),
                   "rng_begin")
        self._host_step += 1
        self._slot = 0

    def reset_step(self, step: int = -1) -> None:
        """Set the step counter (device and host mirror): the next render draws as step + 1."""
        self._host_step = int(step)
        if self._state is not None:
            self._state[1].fill_(int(step))

    def sync_host_step(self) -> int:
        """Re-read the host mirror of the step from the device state (a host sync).  The mirror
        only follows eager renders: replays of a captured graph advance the device step alone."""
        if self._state is not None:
            self._host_step = int(self._state[1].item())
        return self._host_step

    def copy_state_from(self, other: "PhiloxRandom") -> None:
        """Continue from ``other``'s step (same draws from the next render on), its device step
        included (``other`` may have been advanced by graph replays)."""
        self._host_step = other.sync_host_step()
        self._state = None if other._state is None else other._state.clone()

    def key(self, device, nslots: int = 1):
        """(spnerf_rng, the tensor it points at — keep it alive while a kernel may read it)"""
        from ._lib import Rng
        if self._snap is None:
            self.begin_render(device)
        r = Rng(self._snap.data_ptr(), self.ray_offset, self._slot, 0)
        self._slot += nslots
        return r, self._snap

    # draws a host-side caller asks for as tensors (the standalone drop-ins, e.g. sample_3sigma):
    # a generator seeded from (seed, step, slot), not rank-keyed per ray.  The step is the HOST
    # mirror (no device read, so no sync); these fallbacks cannot be captured into a HIP graph
    # (a replay would not advance the mirror and torch generators are host state).
    def _gen(self, device):
        if self._state is not None and not torch.cuda.is_current_stream_capturing():
            self.sync_host_step()   # (graph replays may have moved the device step on)
        g = torch.Generator(device=device)
        g.manual_seed(_mix64(self.seed, max(self._host_step, 0), self._slot) & ((1 << 63) - 1))
        self._slot += 1
        return g

    def rand(self, shape, device):
        return torch.rand(shape, device=device, generator=self._gen(device))

    def noise(self, shape, device, noise_std):
        if noise_std == 0:
            return None
        return torch.randn(shape, device=device, generator=self._gen(device))

    def gt_uniform(self, valid_mask, n, device):
        return self.rand((valid_mask.shape[0], n), device)


def _splitmix64(x: int) -> int:
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


def _mix64(seed: int, step: int, slot: int) -> int:
    """(seed, step, slot) -> 64-bit generator seed; distinct triples do not collide the way a
    linear combination does."""
    return _splitmix64(_splitmix64(_splitmix64(seed & ((1 << 64) - 1)) ^ (step & ((1 << 64) - 1))) ^ slot)


def begin_render(device) -> None:
    """Start of a render_rays call: a keyed on-device source advances its step."""
    src = current_random_source()
    if getattr(src, "on_device", False):
        src.begin_render(device)


def device_key(device, nslots: int = 1):
    """(spnerf_rng, keep-alive) of the current source when it draws on the device, else (None, None)."""
    src = current_random_source()
    if getattr(src, "on_device", False):
        return src.key(device, nslots)
    return None, None


_state = threading.local()


def current_random_source():
    return getattr(_state, "src", None) or _DEFAULT


def set_random_source(src):
    _state.src = src


@contextlib.contextmanager
def random_source(src):
    prev = getattr(_state, "src", None)
    _state.src = src
    try:
        yield src
    finally:
        _state.src = prev


_DEFAULT = TorchRandom()
