"""Shared helpers for the golden-fixture tests (loading, RNG replay, comparison)."""
from __future__ import annotations

import ast
import os
import types

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = ["c1_w512", "c1_w64", "c3_w64", "c3_w512", "c3_test_w64", "beta_w64", "nomap_w64", "fine_w64",
         "fine_sc_guided_w64", "c5_w512"]


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    meta = ast.literal_eval(str(data.pop("meta")))
    data["meta"] = meta
    return data


def dims_of(meta: dict):
    from oracle.weights import ModelDims
    d = dict(meta["dims"])
    d["skips"] = tuple(d["skips"])
    return ModelDims(**d)


def args_of(meta: dict):
    return types.SimpleNamespace(**meta["args"])


def draws_of(data: dict) -> list:
    keys = sorted(k for k in data if k.startswith("rng"))
    return [(k.split("_", 1)[1], data[k]) for k in keys]


class Replay:
    """Random source that hands back the reference's recorded draws in order."""

    def __init__(self, draws: list, to_tensor):
        self.draws = list(draws)
        self.to_tensor = to_tensor
        self.used = 0

    def __call__(self, kind: str, shape: tuple):
        k, arr = self.draws[self.used]
        assert k == kind and tuple(arr.shape) == tuple(shape), (self.used, k, kind, arr.shape, shape)
        self.used += 1
        return self.to_tensor(arr)


def synthetic_rays(n: int, seed: int, far_scale: float = 0.21) -> np.ndarray:
    """JAX_269-like normalised rays (n, 11): origins inside the unit scene box, unit
    directions within ~6 deg of the local down vector at Jacksonville (lat 30.3, lon
    -81.7) expressed in ECEF, near = 0, far ≈ 28 m / 141.2 m, sun_d = (0, 1, 0)
    (JAX_269 JSONs carry sun_elevation = sun_azimuth = 0, satellite_scene.py:449-473)."""
    rng = np.random.default_rng(seed)
    down = np.array([-0.124, 0.855, -0.505])
    down /= np.linalg.norm(down)
    o = rng.uniform(-0.8, 0.8, size=(n, 3))
    d = down + rng.normal(scale=0.05, size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    far = far_scale * rng.uniform(0.95, 1.1, size=n)
    rays = np.zeros((n, 11), np.float64)
    rays[:, 0:3], rays[:, 3:6], rays[:, 7] = o, d, far
    rays[:, 9] = 1.0
    return rays.astype(np.float32)


def projection_weights(shapes: dict, seed: int = 1234) -> dict:
    rng = np.random.default_rng(seed)
    return {k: rng.standard_normal(shapes[k]).astype(np.float32) for k in sorted(shapes)}


def param_projections(names_shapes: list, seed: int = 4321) -> dict:
    rng = np.random.default_rng(seed)
    return {n: rng.standard_normal(s).astype(np.float32) for n, s in names_shapes}


def rel_err(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def assert_close(name, got, ref, rtol=1e-4, atol_frac=1e-5):
    """Element-wise |got-ref| <= rtol*|ref| + atol_frac*max|ref| (the 1e-4 relative fp32
    tolerance of BASELINE.json north_star, with an absolute floor scaled to the tensor)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    bad = np.abs(got - ref) > rtol * np.abs(ref) + atol_frac * scale + 1e-30
    nan_mismatch = np.isnan(got) != np.isnan(ref)
    bad = (bad & ~(np.isnan(got) & np.isnan(ref))) | nan_mismatch
    if bad.any():
        i = np.argmax(np.where(bad, np.abs(got - ref), -1))
        raise AssertionError(f"{name}: {bad.sum()}/{bad.size} out of tol; worst idx {np.unravel_index(i, ref.shape)} "
                             f"got {got.flat[i]!r} ref {ref.flat[i]!r}; rel_err {rel_err(got, ref):.3e}")
