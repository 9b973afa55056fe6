"""Random source of the render path.

The reference draws every random tensor from torch's global generator, in a fixed order
(SURVEY.md §4): stratified jitter ``rand (B,S)`` (rendering.py:143), σ noise ``randn``
per inference call (spnerf.py:122), ``rand (B,S)`` for the predicted-depth window
(rendering.py:35 via :87) and ``rand (B_valid,S)`` for the GT window (:113).

``TorchRandom`` (the default) draws the same tensors with torch on the rays' device; it
skips the σ-noise draw when ``noise_std == 0`` (the product with 0 is exactly 0) and draws
the GT-window ``u`` for every ray, indexed by ray, so no host synchronisation is needed to
count the valid rays.  ``ReplayRandom`` hands back pre-recorded draws (the reference's, in
the parity tests) in the reference's order and shapes.
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
