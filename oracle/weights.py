"""Deterministic SP-NeRF parameter sets — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything under ``oracle/``; the product path never does.

The golden fixtures under ``tests/golden/`` do not ship the (10.8 MB at W=512)
weights.  Instead both the fixture generator and the tests rebuild them from
this documented numpy generator: parameters are visited in the reference's
registration order (= ``SPNeRF.named_parameters()`` order, models/spnerf.py
:162-264) and each one is drawn ``U(-b, b)`` from ONE ``numpy.random.
default_rng(seed)`` stream, with ``b`` the bound of the reference initialiser
for that tensor:

* ``fc_net.*.weight`` and ``sun_v_net.*.weight``: ``sine_init`` bound
  ``sqrt(6/fan_in)`` (spnerf.py:49-53, applied at :251-254);
* ``fc_net.0.weight`` and ``sun_v_net.0.weight``: ``first_layer_sine_init``
  bound ``1/fan_in`` (spnerf.py:56-60, :253,255);
* every other Linear weight and every Linear bias: PyTorch's default
  ``1/sqrt(fan_in)``;
* ``semantic_embedding.weight``: ``N(0,1)`` via ``standard_normal`` with the
  padding row (index C, spnerf.py:191-194) zeroed.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass(frozen=True)
class ModelDims:
    """Construction flags of ``SPNeRF`` (models/__init__.py:6-13)."""
    width: int = 512            # --fc_units (modules/opt.py:43)
    layers: int = 8             # --fc_layers
    skips: tuple = (4,)         # SPNeRF default skips=[4]
    mapping: bool = True        # --mapping (PE on)
    n_freq: int = 10            # mapping_sizes[0]
    sem: bool = False           # --sem
    num_sem_classes: int = 3    # --num_sem_classes
    s_embedding_factor: int = 1
    beta: bool = False          # --beta
    t_dim: int = 4              # --t_embbeding_tau

    @property
    def in_xyz(self) -> int:
        return 2 * self.n_freq * 3 if self.mapping else 3

    @property
    def sem_dim(self) -> int:
        return self.num_sem_classes * self.s_embedding_factor if self.sem else 0

    @property
    def input_size(self) -> int:
        return self.in_xyz + self.sem_dim

    @property
    def n_outputs(self) -> int:
        return 8 + (1 if self.beta else 0) + (self.num_sem_classes if self.sem else 0)


def param_specs(d: ModelDims):
    """[(name, shape, bound_kind)] in registration order (spnerf.py:162-264)."""
    W, H = d.width, d.width // 2
    specs = []
    if d.sem:
        specs.append(("semantic_embedding.weight", (d.num_sem_classes + 1, d.sem_dim), "embed"))
    for i in range(d.layers):
        fan = d.input_size if i == 0 else (W + d.input_size if i in d.skips else W)
        specs.append((f"fc_net.{2*i}.weight", (W, fan), "first" if i == 0 else "sine"))
        specs.append((f"fc_net.{2*i}.bias", (W,), "default"))
    specs += [("sigma_from_xyz.0.weight", (1, W), "default"), ("sigma_from_xyz.0.bias", (1,), "default"),
              ("feats_from_xyz.weight", (W, W), "default"), ("feats_from_xyz.bias", (W,), "default")]
    if d.sem:
        specs += [("logit_from_label.0.weight", (H, W), "default"), ("logit_from_label.0.bias", (H,), "default"),
                  ("logit_from_label.2.weight", (d.num_sem_classes, H), "default"),
                  ("logit_from_label.2.bias", (d.num_sem_classes,), "default")]
    specs += [("rgb_from_xyzdir.0.weight", (H, W), "default"), ("rgb_from_xyzdir.0.bias", (H,), "default"),
              ("rgb_from_xyzdir.2.weight", (3, H), "default"), ("rgb_from_xyzdir.2.bias", (3,), "default")]
    sun_fans = [W + 3, H, H, H]
    sun_outs = [H, H, H, 1]
    for j in range(4):
        specs.append((f"sun_v_net.{2*j}.weight", (sun_outs[j], sun_fans[j]), "first" if j == 0 else "sine"))
        specs.append((f"sun_v_net.{2*j}.bias", (sun_outs[j],), "default"))
    specs += [("sky_color.0.weight", (H, 3), "default"), ("sky_color.0.bias", (H,), "default"),
              ("sky_color.2.weight", (3, H), "default"), ("sky_color.2.bias", (3,), "default")]
    if d.beta:
        specs += [("beta_from_xyz.0.weight", (H, d.t_dim + W), "default"), ("beta_from_xyz.0.bias", (H,), "default"),
                  ("beta_from_xyz.2.weight", (1, H), "default"), ("beta_from_xyz.2.bias", (1,), "default")]
    return specs


def _fan_in(name: str, shape, specs_by_name) -> int:
    if name.endswith(".bias"):
        return specs_by_name[name[:-5] + ".weight"][1]
    return shape[-1]


def make_weights(d: ModelDims, seed: int = 0) -> "dict[str, np.ndarray]":
    """Deterministic float32 parameters, keyed by reference state-dict name."""
    rng = np.random.default_rng(seed)
    specs = param_specs(d)
    by_name = {n: s for n, s, _ in specs}
    out = {}
    for name, shape, kind in specs:
        if kind == "embed":
            w = rng.standard_normal(shape).astype(np.float32)
            w[d.num_sem_classes] = 0.0
        else:
            fan = _fan_in(name, shape, by_name)
            b = {"sine": math.sqrt(6.0 / fan), "first": 1.0 / fan}.get(kind, 1.0 / math.sqrt(fan))
            w = rng.uniform(-b, b, size=shape).astype(np.float32)
        out[name] = w
    return out
