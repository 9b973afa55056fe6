"""RPC ray generation, restated in numpy — TEST INFRASTRUCTURE ONLY (parity checker of the
GPU ray generator, spnerf_rpc_rays).

Third-party dependency restated: ``rpcm`` (RPCModel / localization), which the reference uses
at datasets/satellite_scene.py:43,48 through ``rpcm.RPCModel(d["rpc"], dict_format="rpcm")``
(:192) and ``utils.rescale_rpc`` (modules/utils.py:59-77).  rpcm is neither vendored nor
version-pinned (requirements.txt:2 lists a bare ``rpcm``), so its result is **parity-unpinned
against rpcm itself**; what pins this restatement is (1) the round trip
project(localize(c, r, h)) == (c, r) to 1e-9 normalised units, which any converged rpcm
localization also satisfies, and (2) the reference's own get_rays / normalize_rays /
geodetic_to_ecef / get_sun_dirs run on top of it (tests/golden/gen_golden.py::rpc_rays).

Algorithm (rpcm's published RPC00B model):
* projection ground→image: col = P_cn(lat, lon, alt) / P_cd(...), row likewise, on normalised
  coordinates, with the 20-term monomial order
  1, L, P, H, LP, LH, PH, L², P², H², PLH, L³, LP², LH², L²P, P³, PH², L²H, P²H, H³
  (L = lon, P = lat, H = alt);
* localization image→ground: rpcm's iterative scheme — project the current estimate and two
  offset points (lon + EPS, lat + EPS), decompose the image-space residual on the two offset
  vectors, step, EPS = 2 on the first iteration then 0.1, until the squared normalised
  residual < 1e-18.
"""
from __future__ import annotations

import numpy as np

KEYS = ("row_offset", "col_offset", "lat_offset", "lon_offset", "alt_offset",
        "row_scale", "col_scale", "lat_scale", "lon_scale", "alt_scale")


def poly(c, lat, lon, alt):
    x, y, z = lat, lon, alt
    return (c[0] + c[1] * y + c[2] * x + c[3] * z + c[4] * y * x + c[5] * y * z + c[6] * x * z + c[7] * y * y
            + c[8] * x * x + c[9] * z * z + c[10] * x * y * z + c[11] * y * y * y + c[12] * y * x * x
            + c[13] * y * z * z + c[14] * y * y * x + c[15] * x * x * x + c[16] * x * z * z + c[17] * y * y * z
            + c[18] * x * x * z + c[19] * z * z * z)


class RPC:
    def __init__(self, d: dict, downscale: float = 1.0):
        for k in KEYS:
            setattr(self, k, float(d[k]))
        self.row_num, self.row_den = np.array(d["row_num"], float), np.array(d["row_den"], float)
        self.col_num, self.col_den = np.array(d["col_num"], float), np.array(d["col_den"], float)
        if downscale != 1.0:          # utils.rescale_rpc(rpc, 1/downscale), modules/utils.py:59-77
            a = 1.0 / float(downscale)
            self.row_scale *= a
            self.col_scale *= a
            self.row_offset *= a
            self.col_offset *= a

    def projection_n(self, lat, lon, alt):
        col = poly(self.col_num, lat, lon, alt) / poly(self.col_den, lat, lon, alt)
        row = poly(self.row_num, lat, lon, alt) / poly(self.row_den, lat, lon, alt)
        return col, row

    def projection(self, lon, lat, alt):
        c, r = self.projection_n((lat - self.lat_offset) / self.lat_scale, (lon - self.lon_offset) / self.lon_scale,
                                 (alt - self.alt_offset) / self.alt_scale)
        return c * self.col_scale + self.col_offset, r * self.row_scale + self.row_offset

    def localization(self, col, row, alt):
        cn = (np.asarray(col, float) - self.col_offset) / self.col_scale
        rn = (np.asarray(row, float) - self.row_offset) / self.row_scale
        an = (np.asarray(alt, float) - self.alt_offset) / self.alt_scale
        lon = -np.ones_like(cn)
        lat = -np.ones_like(cn)
        eps = 2.0
        for _ in range(101):
            x0, y0 = self.projection_n(lat, lon, an)
            if np.all((x0 - cn) ** 2 + (y0 - rn) ** 2 < 1e-18):
                break
            x1, y1 = self.projection_n(lat, lon + eps, an)
            x2, y2 = self.projection_n(lat + eps, lon, an)
            e1x, e1y, e2x, e2y = x1 - x0, y1 - y0, x2 - x0, y2 - y0
            ux, uy = cn - x0, rn - y0
            a1 = (ux * e1x + uy * e1y) / (e1x * e1x + e1y * e1y)
            a2 = (ux * e2x + uy * e2y) / (e2x * e2x + e2y * e2y)
            lon = lon + a1 * eps
            lat = lat + a2 * eps
            eps = 0.1
        else:
            raise RuntimeError("localization did not converge")
        return lon * self.lon_scale + self.lon_offset, lat * self.lat_scale + self.lat_offset


def geodetic_to_ecef(lat, lon, alt):
    """modules/utils.py:80-100 (WGS-84)."""
    a, b = 6378137.0, 6356752.314245
    e2 = 1 - (b ** 2 / a ** 2)
    la, lo = np.radians(lat), np.radians(lon)
    n = a / np.sqrt(1 - e2 * np.sin(la) ** 2)
    return ((n + alt) * np.cos(la) * np.cos(lo), (n + alt) * np.cos(la) * np.sin(lo),
            ((b ** 2 / a ** 2) * n + alt) * np.sin(la))


def get_rays(cols, rows, rpc: RPC, min_alt, max_alt) -> np.ndarray:
    """datasets/satellite_scene.py:21-68 → (n, 8) float32 [o, d, near, far]."""
    lon, lat = rpc.localization(cols, rows, np.full(len(cols), float(max_alt)))
    near = np.stack(geodetic_to_ecef(lat, lon, np.full(len(cols), float(max_alt))), 1)
    lon, lat = rpc.localization(cols, rows, np.full(len(cols), float(min_alt)))
    far = np.stack(geodetic_to_ecef(lat, lon, np.full(len(cols), float(min_alt))), 1)
    d = far - near
    nrm = np.linalg.norm(d, axis=1)
    return np.hstack([near, d / nrm[:, None], np.zeros((len(cols), 1)), nrm[:, None]]).astype(np.float32)


def normalize_rays(rays: np.ndarray, center, rng) -> np.ndarray:
    """satellite_scene.py:415-425, in fp32 (center and range are float32 tensors there)."""
    r = rays.astype(np.float32).copy()
    c = np.asarray(center, np.float32)
    rg = np.float32(rng)
    r[:, 0:3] = (r[:, 0:3] - c) / rg
    r[:, 6:8] = r[:, 6:8] / rg
    return r


def sun_dirs(elev_deg, azim_deg, n) -> np.ndarray:
    """satellite_scene.py:449-473."""
    el, az = np.radians(elev_deg), np.radians(azim_deg)
    v = np.array([np.sin(az) * np.cos(el), np.cos(az) * np.cos(el), np.sin(el)])
    return np.tile(v, (n, 1)).astype(np.float32)
