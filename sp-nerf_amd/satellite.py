"""Satellite camera rays on the GPU — the ray generator of datasets/satellite_scene.py.

Drop-ins for ``get_rays`` (:21-68), ``SatelliteSceneDataset.normalize_rays`` (:415-425),
``get_sun_dirs`` (:449-473) and ``utils.rescale_rpc`` (modules/utils.py:59-77), plus
``image_rays``, which fuses all of them into ONE kernel launch per image
(``spnerf_rpc_rays``, csrc/rays.hip): rpcm-style fp64 localization at max/min altitude,
WGS-84 ECEF, fp32 quantisation, fp32 normalisation, sun direction.  The reference runs this
on the CPU with rpcm at dataset construction; at 4k×4k (config 5, 16.8 M rays) that is the
bottleneck this removes.

Camera metadata of the reference's JAX_269 scene (RPCs, sizes, altitude bounds, sun angles,
scene.loc) ships as data in ``data/jax269_cameras.json``.
"""
from __future__ import annotations

import ctypes
import json
import math
import os

import numpy as np
import torch

from . import _lib

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "jax269_cameras.json")
_OFF = ("row_offset", "col_offset", "lat_offset", "lon_offset", "alt_offset",
        "row_scale", "col_scale", "lat_scale", "lon_scale", "alt_scale")


class RPCModel:
    """RPC00B camera (rpcm.RPCModel(d, dict_format="rpcm") fields)."""

    def __init__(self, d: dict):
        for k in _OFF:
            setattr(self, k, float(d[k]))
        self.row_num, self.row_den = list(map(float, d["row_num"])), list(map(float, d["row_den"]))
        self.col_num, self.col_den = list(map(float, d["col_num"])), list(map(float, d["col_den"]))

    def packed(self) -> "ctypes.Array":
        vals = [getattr(self, k) for k in _OFF] + self.row_num + self.row_den + self.col_num + self.col_den
        return (ctypes.c_double * 90)(*vals)


def rescale_rpc(rpc: RPCModel, alpha: float) -> RPCModel:
    """modules/utils.py:59-77."""
    import copy
    r = copy.copy(rpc)
    r.row_scale *= float(alpha)
    r.col_scale *= float(alpha)
    r.row_offset *= float(alpha)
    r.col_offset *= float(alpha)
    return r


def load_cameras(path: str = DATA) -> dict:
    with open(path) as f:
        return json.load(f)


def scene_normalisation(loc: dict):
    """center and range of satellite_scene.py:118-124 (float32 tensors there)."""
    center = np.array([float(loc["X_offset"]), float(loc["Y_offset"]), float(loc["Z_offset"])], np.float32)
    rng = np.float32(max(float(loc["X_scale"]), float(loc["Y_scale"]), float(loc["Z_scale"])))
    return center, rng


def sun_direction(elev_deg: float, azim_deg: float) -> np.ndarray:
    el, az = math.radians(elev_deg), math.radians(azim_deg)
    return np.array([math.sin(az) * math.cos(el), math.cos(az) * math.cos(el), math.sin(el)], np.float64)


def _launch(rpc: RPCModel, min_alt, max_alt, out, stride, rect=None, pixels=None, center=None, rng=1.0, sun=None):
    L = _lib.lib()
    cen = (ctypes.c_float * 3)(*[float(v) for v in center]) if center is not None else None
    sn = (ctypes.c_float * 3)(*[float(v) for v in np.asarray(sun, np.float64).astype(np.float32)]) if sun is not None else None
    r0, c0, nr, nc = rect if rect is not None else (0, 0, 0, 0)
    n_pix = pixels.shape[0] if pixels is not None else 0
    _lib.check(L.spnerf_rpc_rays(rpc.packed(), 1.0, float(min_alt), float(max_alt), r0, c0, nr, nc, _lib.ptr(pixels),
                                 n_pix, cen, float(rng), sn, _lib.ptr(out), stride, _lib.stream_of(out)), "rpc_rays")


def get_rays(cols, rows, rpc: RPCModel, min_alt, max_alt, device="cuda") -> torch.Tensor:
    """satellite_scene.py:21-68: (n, 8) float32 [o (ECEF), d, near = 0, far = ‖far − near‖]."""
    pix = torch.as_tensor(np.stack([np.asarray(cols), np.asarray(rows)], 1).astype(np.int32), device=device).contiguous()
    out = torch.empty(pix.shape[0], 8, device=device)
    _lib.require_device(out)
    _launch(rpc, min_alt, max_alt, out, 8, pixels=pix)
    return out


def normalize_rays(rays: torch.Tensor, center, rng) -> torch.Tensor:
    """satellite_scene.py:415-425 (in place, fp32)."""
    c = torch.as_tensor(np.asarray(center, np.float32), device=rays.device)
    r = torch.as_tensor(np.float32(rng), device=rays.device)
    rays[:, 0:3] -= c
    rays[:, 0:3] /= r
    rays[:, 6:8] /= r
    return rays


def get_sun_dirs(sun_elevation_deg, sun_azimuth_deg, n_rays, device="cuda") -> torch.Tensor:
    """satellite_scene.py:449-473."""
    v = torch.tensor(sun_direction(sun_elevation_deg, sun_azimuth_deg).astype(np.float32), device=device)
    return v.expand(n_rays, 3).contiguous()


def image_rays(meta: dict, img_downscale: float, loc: dict, crop=None, device="cuda") -> torch.Tensor:
    """All rays of one image (row-major, satellite_scene.py:186-221) as (n, 11) normalised
    [o, d, near, far, sun] — one fused kernel.  crop = (row0, col0, n_rows, n_cols)."""
    h, w = int(meta["height"] // img_downscale), int(meta["width"] // img_downscale)
    rpc = rescale_rpc(RPCModel(meta["rpc"]), 1.0 / img_downscale)
    rect = crop if crop is not None else (0, 0, h, w)
    center, rng = scene_normalisation(loc)
    out = torch.empty(rect[2] * rect[3], 11, device=device)
    _lib.require_device(out)
    _launch(rpc, meta["min_alt"], meta["max_alt"], out, 11, rect=rect, center=center, rng=rng,
            sun=sun_direction(float(meta["sun_elevation"]), float(meta["sun_azimuth"])))
    return out
