"""Benchmark scene of the JAX_214 shape.

JAX_214 imagery is not shipped with the reference (only DFC2019_269 is), so, as SURVEY §8d
prescribes, the JAX_269 RPC cameras stand in for it: three views (README's
``JAX_214_3_imgs``: JAX_269_006 / 007 / 011), rays generated on the GPU by the RPC ray
generator (satellite.image_rays: get_rays + normalize_rays + get_sun_dirs of
datasets/satellite_scene.py) at the requested ``img_downscale``, in the dataset's order
(images concatenated, pixels row-major; satellite_scene.py:186-221).  The JSONs carry
sun_elevation = sun_azimuth = 0, hence sun_d = (0, 1, 0).

Colour targets: at img_downscale 4 the REAL JAX_269 images (data/jax269_rgb_ds4.npz, made from
the reference's GeoTIFFs by tools/make_rgb_targets.py the way its dataset downsamples them,
satellite_scene.py:71-86); at other scales (no GeoTIFF I/O on the GPU box) a smooth synthetic
albedo field of the ray's ground point.  Depth priors valid on ~68 % of the rays (JAX_269's
2D-point coverage 438,256 / 644,709) with GT depth far·U(0.3, 0.7) and std (1-corr)·0.05+1e-4;
semantic labels {0, 1, 2, -100} with fixed frequencies.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from .satellite import image_rays, load_cameras

VIEWS = ("JAX_269_006_RGB", "JAX_269_007_RGB", "JAX_269_011_RGB")


@dataclass
class Scene:
    rays: torch.Tensor        # (N, 11) float32 [o(3), d(3), near, far, sun(3)]
    rgbs: torch.Tensor        # (N, 3)
    depths: torch.Tensor      # (N, 2) [depth, correlation]
    valid_depth: torch.Tensor  # (N,) int64
    depth_std: torch.Tensor   # (N,)
    sems: torch.Tensor        # (N,) int64 in {0, 1, 2, -100}
    view_sizes: list
    rgb_source: str = "synthetic"

    def to(self, device):
        return Scene(*(getattr(self, f).to(device) for f in ("rays", "rgbs", "depths", "valid_depth", "depth_std", "sems")),
                     self.view_sizes, self.rgb_source)


def real_rgbs(views, img_downscale: float):
    """The views' real pixels (N, 3) in the rays' order, or None when not shipped at this scale."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", f"jax269_rgb_ds{int(img_downscale)}.npz")
    if img_downscale != int(img_downscale) or not os.path.exists(path):
        return None
    with np.load(path, allow_pickle=False) as z:
        if not all(v in z.files for v in views):
            return None
        return torch.tensor(np.concatenate([z[v] for v in views]))


def synthetic_scene(img_downscale: float = 4.0, views=VIEWS, seed: int = 0, device="cuda") -> Scene:
    cams = load_cameras()
    rays, sizes = [], []
    for v in views:
        meta = cams["images"][v]
        rays.append(image_rays(meta, img_downscale, cams["scene_loc"], device=device))
        sizes.append((int(meta["height"] // img_downscale), int(meta["width"] // img_downscale)))
    rays = torch.cat(rays)
    n = rays.shape[0]
    g = torch.Generator(device="cpu").manual_seed(seed)
    rgbs = real_rgbs(views, img_downscale)
    source = "real JAX_269 RGB" if rgbs is not None else "synthetic"
    if rgbs is not None:
        assert rgbs.shape[0] == n, (rgbs.shape, n)
        rgbs = rgbs.to(rays.device)
    else:
        mid = rays[:, 0:3] + 0.5 * rays[:, 7:8] * rays[:, 3:6]
        gx, gy = mid[:, 0] + mid[:, 2], mid[:, 1]
        rgbs = torch.stack([0.45 + 0.3 * torch.sin(9 * gx), 0.5 + 0.25 * torch.cos(7 * gy),
                            0.4 + 0.2 * torch.sin(5 * (gx + gy))], 1).clamp(0, 1)
    valid = (torch.rand(n, generator=g) < 438256 / 644709).long()
    gt = rays[:, 7].cpu() * (0.3 + 0.4 * torch.rand(n, generator=g))
    corr = 0.2 + 0.8 * torch.rand(n, generator=g)
    std = (1.0 - corr) * 0.05 + 1e-4
    sems = torch.multinomial(torch.tensor([0.45, 0.3, 0.15, 0.1]), n, replacement=True, generator=g)
    sems = torch.where(sems == 3, torch.full_like(sems, -100), sems)
    dev = rays.device
    return Scene(rays, rgbs.float(), torch.stack([gt, corr], 1).float().to(dev), valid.to(dev), std.float().to(dev),
                 sems.to(dev), sizes, source)
