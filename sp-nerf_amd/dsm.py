"""DSM extraction from a rendered depth image: drop-ins for
``SatelliteSceneDataset.get_latlonalt_from_nerf_prediction`` / ``get_dsm_from_nerf_prediction``
(datasets/satellite_scene.py:475-568) and the MAE of ``utils.compute_mae_and_save_dsm_diff``
(modules/utils.py:142-245), on the GPU (csrc/dsm.hip, fp64).

The reference converts the point cloud on the CPU (numpy + pyproj) and rasterises it with
plyflatten; here the lat/lon/alt, UTM and rasterisation run as three kernel launches over the
render's rays, and only the DSM (a few MB) comes back to the host.  pyproj and plyflatten are
not installed here: the UTM projection is the transverse-Mercator algorithm PROJ's utm uses
(Krüger series) and the rasteriser plyflatten's documented behaviour — both parity unpinned
(oracle/dsm_ref.py); lat/lon/alt is pinned to the reference's own function.  The MAE follows the
reference's no-dsmr branch (registration by the mean Z offset, utils.py:197-201); the GDAL crop
is the array window of the ROI grid.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import _lib

_ZONE_LETTERS = "CDEFGHJKLMNPQRSTUVWXX"


def utm_zone(lat: float, lon: float):
    """utm.latlon_to_zone_number / latitude_to_zone_letter (the reference's zone of the first
    point, utils.py:133-134)."""
    if 56 <= lat < 64 and 3 <= lon < 12:
        n = 32
    elif 72 <= lat <= 84 and lon >= 0 and lon < 42:
        n = 31 if lon < 9 else 33 if lon < 21 else 35 if lon < 33 else 37
    else:
        n = int((lon + 180) / 6) + 1
    letter = _ZONE_LETTERS[int(lat + 80) >> 3] if -80 <= lat <= 84 else None
    return n, letter


def _points(rays: torch.Tensor, depth: torch.Tensor, center, rng, zone=1, south=False, lla=True, ena=False):
    _lib.require_device(rays, depth)
    rays = rays.contiguous().float()
    depth = depth.reshape(-1).contiguous().float()
    n = rays.shape[0]
    if depth.shape[0] != n or rays.dim() != 2 or rays.shape[1] < 6:
        raise ValueError("rays must be (n, >=6) and depth (n,) or (n, 1)")
    cen = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(center, np.float32).reshape(3)])
    out_lla = torch.empty(n, 3, dtype=torch.float64, device=rays.device) if lla else None
    out_ena = torch.empty(n, 3, dtype=torch.float64, device=rays.device) if ena else None
    _lib.check(_lib.lib().spnerf_dsm_points(_lib.ptr(rays), rays.shape[1], n, _lib.ptr(depth), cen,
                                           float(np.float32(rng)), int(zone), 1 if south else 0, _lib.ptr(out_lla),
                                           _lib.ptr(out_ena), _lib.stream_of(rays)), "dsm_points")
    return out_lla, out_ena


def get_latlonalt_from_nerf_prediction(rays: torch.Tensor, depth: torch.Tensor, center, rng):
    """satellite_scene.py:475-505: numpy (lats, lons, alts) of the predicted points.  ``center``
    and ``rng`` are the scene's normalisation (SatelliteSceneDataset.center / .range)."""
    lla, _ = _points(rays, depth, center, rng)
    lla = lla.cpu().numpy()
    return lla[:, 0], lla[:, 1], lla[:, 2]


def get_dsm_from_nerf_prediction(rays: torch.Tensor, depth: torch.Tensor, center, rng, dsm_path=None, roi_txt=None,
                                 resolution=0.5, radius=1, sigma=float("inf")):
    """satellite_scene.py:507-568: the (ysize, xsize, 1) float64 DSM of the predicted points,
    NaN where no point lands.  ``roi_txt`` (the lidar ROI file: xoff, yoff, size, resolution)
    fixes the grid like the reference; otherwise the cloud's bounds at ``resolution``.  With
    ``dsm_path`` the DSM is written as a float32 TIFF (PIL; no GeoTIFF tags — rasterio is not
    installed) with its grid in ``<dsm_path>.txt`` (xoff, yoff-of-the-top-row, xsize, ysize,
    resolution, UTM zone)."""
    lla, _ = _points(rays[:1], depth.reshape(-1)[:1], center, rng)
    lat0, lon0 = float(lla[0, 0]), float(lla[0, 1])
    zone, letter = utm_zone(lat0, lon0)
    # the reference asks pyproj for "+proj=utm +zone=<n><letter>" without +south; PROJ reads the
    # zone number only, so the northern false northing applies everywhere (kept)
    _, ena = _points(rays, depth, center, rng, zone=zone, south=False, lla=False, ena=True)
    if roi_txt is not None:
        meta = np.loadtxt(roi_txt)
        xoff, yoff = float(meta[0]), float(meta[1])
        xsize = ysize = int(meta[2])
        res = float(meta[3])
        yoff += ysize * res
    else:
        lo = ena[:, :2].amin(0).cpu().numpy()
        hi = ena[:, :2].amax(0).cpu().numpy()
        res = float(resolution)
        xoff = math.floor(lo[0] / res) * res
        xsize = int(1 + math.floor((hi[0] - xoff) / res))
        yoff = math.ceil(hi[1] / res) * res
        ysize = int(1 - math.floor((lo[1] - yoff) / res))
    dsm = rasterize(ena, xoff, yoff, res, xsize, ysize, radius=radius, sigma=sigma)
    out = dsm.cpu().numpy()[:, :, None]
    if dsm_path is not None:
        from PIL import Image
        os.makedirs(os.path.dirname(dsm_path) or ".", exist_ok=True)
        Image.fromarray(out[:, :, 0].astype(np.float32), mode="F").save(dsm_path)
        with open(dsm_path + ".txt", "w") as f:
            f.write(f"{xoff:.6f}\n{yoff:.6f}\n{xsize}\n{ysize}\n{res:.6f}\n{zone}{letter or ''}\n")
    return out


def rasterize(ena: torch.Tensor, xoff, yoff, resolution, xsize, ysize, radius=1, sigma=float("inf")) -> torch.Tensor:
    """plyflatten(cloud, xoff, yoff, resolution, xsize, ysize, radius, sigma) on the device:
    ``ena`` (n, 3) float64 easting / northing / altitude -> (ysize, xsize) float64."""
    _lib.require_device(ena)
    ena = ena.contiguous().double()
    acc = torch.empty(2, ysize, xsize, dtype=torch.float64, device=ena.device)
    dsm = torch.empty(ysize, xsize, dtype=torch.float64, device=ena.device)
    _lib.check(_lib.lib().spnerf_dsm_rasterize(_lib.ptr(ena), ena.shape[0], float(xoff), float(yoff), float(resolution),
                                              int(xsize), int(ysize), int(radius), float(sigma), _lib.ptr(acc),
                                              _lib.ptr(dsm), _lib.stream_of(ena)), "dsm_rasterize")
    return dsm


def dsm_mae(pred_dsm, gt_dsm) -> float:
    """The MAE of utils.compute_mae_and_save_dsm_diff on arrays already on the ground truth's
    grid, along the reference's no-dsmr branch (utils.py:197-201: shift by the mean Z offset)."""
    pred = np.asarray(pred_dsm, np.float64).reshape(np.asarray(gt_dsm).shape)
    gt = np.asarray(gt_dsm, np.float64)
    rp = pred + np.nanmean(gt - pred)
    return float(np.nanmean(np.abs(rp - gt)))
