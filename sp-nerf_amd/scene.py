"""Synthetic satellite scene of the JAX_214 shape (benchmark / smoke data).

JAX_214 imagery is not shipped with the reference (only DFC2019_269 is), so the benchmark
uses synthetic rays with the layout of ``SatelliteSceneDataset`` (datasets/satellite_scene.py
:167-221): per view, one ray per pixel in row-major order, ``[o(3), d(3), near, far, sun(3)]``
in the normalised ECEF frame (``scene.loc`` range 141.21875), near = 0 and far = altitude span
/ cos(off-nadir).  Each view is an off-nadir pushbroom-like affine camera over the unit AOI
(3 train views, README's ``JAX_214_3_imgs``; 813×793 px like JAX_269_006 at ds=1).  Targets:
a smooth synthetic albedo field; depth priors (valid ~68 %, as JAX_269's 2D-point coverage
438,256 / 644,709) and semantic labels {0,1,2,-100} for the config-3 flags.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

RANGE = 141.21875          # max(X,Y,Z)_scale of JAX_269 scene.loc
ALT_SPAN_M = 28.0          # max_alt - min_alt of the JAX JSONs (-2 .. -30 m)
# local frame at Jacksonville (lat 30.3, lon -81.7) in ECEF
_LAT, _LON = math.radians(30.3), math.radians(-81.7)
UP = np.array([math.cos(_LAT) * math.cos(_LON), math.cos(_LAT) * math.sin(_LON), math.sin(_LAT)])
EAST = np.array([-math.sin(_LON), math.cos(_LON), 0.0])
NORTH = np.cross(UP, EAST)


@dataclass
class Scene:
    rays: torch.Tensor        # (N, 11) float32
    rgbs: torch.Tensor        # (N, 3)
    depths: torch.Tensor      # (N, 2) [depth, correlation]
    valid_depth: torch.Tensor  # (N,) int64
    depth_std: torch.Tensor   # (N,)
    sems: torch.Tensor        # (N,) int64 in {0, 1, 2, -100}
    view_sizes: list


def sun_direction(elev_deg: float, azim_deg: float) -> np.ndarray:
    """get_sun_dirs (satellite_scene.py:449-473) for one image, in the local frame."""
    el, az = math.radians(elev_deg), math.radians(azim_deg)
    return np.array([math.sin(az) * math.cos(el), math.cos(az) * math.cos(el), math.sin(el)])


def synthetic_scene(img_downscale: float = 4.0, n_views: int = 3, height: int = 813, width: int = 793,
                    seed: int = 0) -> Scene:
    rng = np.random.default_rng(seed)
    h, w = int(height // img_downscale), int(width // img_downscale)
    views = [(8.0, 30.0), (17.0, 160.0), (26.0, 280.0)][:n_views]
    rays, rgbs, sizes = [], [], []
    for vi, (theta_deg, phi_deg) in enumerate(views):
        th, ph = math.radians(theta_deg), math.radians(phi_deg)
        d = -math.cos(th) * UP + math.sin(th) * (math.cos(ph) * EAST + math.sin(ph) * NORTH)
        d = d / np.linalg.norm(d)
        r, c = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")          # row-major pixels
        ge = (c.reshape(-1) + 0.5) / w * 1.6 - 0.8
        gn = 0.8 - (r.reshape(-1) + 0.5) / h * 1.6
        far = (ALT_SPAN_M / RANGE) / math.cos(th)
        top = -2.0 / RANGE
        o = ge[:, None] * EAST + gn[:, None] * NORTH + top * UP - d * 0.0
        sun = sun_direction(60.0, 140.0)
        sun_ecef = sun[0] * EAST + sun[1] * NORTH + sun[2] * UP
        v = np.zeros((h * w, 11), np.float64)
        v[:, 0:3], v[:, 3:6], v[:, 7], v[:, 8:11] = o, d, far, sun_ecef
        rays.append(v.astype(np.float32))
        # smooth albedo field of the ground point hit at mid depth
        gx, gy = ge + 0.5 * far * d @ EAST, gn + 0.5 * far * d @ NORTH
        col = np.stack([0.45 + 0.3 * np.sin(7 * gx + 1.3 * vi), 0.5 + 0.25 * np.cos(5 * gy), 0.4 + 0.2 * np.sin(3 * (gx + gy))], 1)
        rgbs.append(np.clip(col, 0, 1).astype(np.float32))
        sizes.append((h, w))
    rays = np.concatenate(rays)
    rgbs = np.concatenate(rgbs)
    n = rays.shape[0]
    valid = (rng.uniform(size=n) < 438256 / 644709).astype(np.int64)
    gt = (rays[:, 7] * rng.uniform(0.3, 0.7, size=n)).astype(np.float32)
    corr = rng.uniform(0.2, 1.0, size=n).astype(np.float32)
    std = ((1.0 - corr) * 0.05 + 1e-4).astype(np.float32)
    sems = rng.choice([0, 1, 2, -100], size=n, p=[0.45, 0.3, 0.15, 0.1]).astype(np.int64)
    return Scene(torch.tensor(rays), torch.tensor(rgbs), torch.tensor(np.stack([gt, corr], 1)), torch.tensor(valid),
                 torch.tensor(std), torch.tensor(sems), sizes)
