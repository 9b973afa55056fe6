"""Real RGB targets for the PSNR-parity runs: the reference's JAX_269 GeoTIFFs, downscaled the
way the reference's dataset does it (datasets/satellite_scene.py:71-86,
load_tensor_from_rgb_geotiff: /255, torchvision Resize to (h // ds, w // ds) with BILINEAR on a
tensor — torchvision 0.8 (requirements.txt, torch 1.7.1) interpolates tensors without
antialiasing, i.e. F.interpolate(mode="bilinear", align_corners=False)), pixels in row-major
order like its rays.  Runs in the build container only (reads /root/reference/Dataset with PIL
instead of rasterio, which is absent); writes sp-nerf_amd/data/jax269_rgb_ds4.npz.

    python tools/make_rgb_targets.py [--ref /root/reference] [--ds 4]
"""
import argparse
import os

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VIEWS = ("JAX_269_006_RGB", "JAX_269_007_RGB", "JAX_269_011_RGB", "JAX_269_023_RGB")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--ds", type=int, default=4)
    a = ap.parse_args()
    out = {}
    for v in VIEWS:
        img = np.asarray(Image.open(os.path.join(a.ref, "Dataset", "DFC2019_269", "RGB", "JAX_269", v + ".tif")))
        img = img.astype(np.float64) / 255.0                                  # (h, w, 3)
        h, w = img.shape[0] // a.ds, img.shape[1] // a.ds
        t = torch.tensor(np.transpose(img, (2, 0, 1)), dtype=torch.float32)[None]  # torch.Tensor(img): fp32
        t = torch.nn.functional.interpolate(t, size=(h, w), mode="bilinear", align_corners=False)[0]
        out[v] = t.permute(1, 2, 0).reshape(-1, 3).numpy().astype(np.float32)  # (h*w, 3) row-major
        out[v + "|hw"] = np.array([h, w])
        print(v, (h, w), float(out[v].mean()))
    path = os.path.join(ROOT, "sp-nerf_amd", "data", f"jax269_rgb_ds{a.ds}.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
