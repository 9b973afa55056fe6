"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's DSM extraction, the checker for
csrc/dsm.hip.  Only tests/ may import it.

  * ecef_to_latlon      — modules/utils.py:103-122 (ecef_to_latlon_custom), pinned to the
                          reference's own function through tests/golden/dsm_latlon.npz
                          (gen_golden.py dsm_latlon: datasets/satellite_scene.py:475-505 run on
                          real JAX_269 rays);
  * utm_zone / utm      — modules/utils.py:125-139 calls pyproj ("+proj=utm +zone=<n><l>") and
                          utm.latlon_to_zone_number / latitude_to_zone_letter; neither package is
                          installed, so this is the published transverse-Mercator algorithm
                          (Krüger's series in n to 6th order, as PROJ's utm / etmerc) and the utm
                          package's zone rules: PARITY UNPINNED beyond known-answer values;
  * rasterize           — satellite_scene.py:547 plyflatten(cloud, xoff, yoff, resolution,
                          xsize, ysize, radius=1, sigma=inf); the plyflatten package (s2p's
                          rasteriser) is absent: restated as documented — each point adds to the
                          (2r+1)^2 cells around its cell (floor((x - xoff)/res), floor((yoff -
                          y)/res)) with weight exp(-d^2 / 2 sigma^2), a cell is the weighted mean,
                          NaN when empty: PARITY UNPINNED;
  * dsm_grid            — the grid bounds of satellite_scene.py:524-538 (ROI file or the cloud's).
"""
import math

import numpy as np

A_WGS84 = 6378137.0
F_WGS84 = 1.0 / 298.257223563


def ecef_to_latlon(x, y, z):
    """modules/utils.py:103-122, float64 numpy."""
    a = 6378137.0
    e = 8.1819190842622e-2
    asq, esq = a ** 2, e ** 2
    b = np.sqrt(asq * (1 - esq))
    bsq = b ** 2
    ep = np.sqrt((asq - bsq) / bsq)
    p = np.sqrt(x ** 2 + y ** 2)
    th = np.arctan2(a * z, b * p)
    lon = np.arctan2(y, x)
    lat = np.arctan2(z + ep ** 2 * b * np.sin(th) ** 3, p - esq * a * np.cos(th) ** 3)
    N = a / np.sqrt(1 - esq * np.sin(lat) ** 2)
    alt = p / np.cos(lat) - N
    return lat * 180 / np.pi, lon * 180 / np.pi, alt


def latlonalt_from_prediction(rays, depth, center, rng):
    """datasets/satellite_scene.py:475-505: rays (n, >=6) and depth (n,) in the normalised scene,
    in double, x = o + d·depth, × range + center, then ecef_to_latlon."""
    rays = np.asarray(rays, np.float64)
    depth = np.asarray(depth, np.float64).reshape(-1, 1)
    xyz = (rays[:, 0:3] + rays[:, 3:6] * depth) * float(rng)
    xyz = xyz + np.asarray(center, np.float64).reshape(1, 3)
    return ecef_to_latlon(xyz[:, 0], xyz[:, 1], xyz[:, 2])


def utm_zone(lat, lon):
    """utm.latlon_to_zone_number (with the Norway / Svalbard exceptions) and
    utm.latitude_to_zone_letter (None outside [-80, 84])."""
    if 56 <= lat < 64 and 3 <= lon < 12:
        n = 32
    elif 72 <= lat <= 84 and lon >= 0:
        n = 31 if lon < 9 else 33 if lon < 21 else 35 if lon < 33 else 37 if lon < 42 else int((lon + 180) / 6) + 1
    else:
        n = int((lon + 180) / 6) + 1
    letters = "CDEFGHJKLMNPQRSTUVWXX"
    letter = letters[int(lat + 80) >> 3] if -80 <= lat <= 84 else None
    return n, letter


def utm(lat, lon, zone, south=False):
    """WGS-84 UTM easting / northing (metres) by Krüger's series to 6th order in n."""
    lat = np.asarray(lat, np.float64)
    lon = np.asarray(lon, np.float64)
    a, f, k0 = A_WGS84, F_WGS84, 0.9996
    n = f / (2 - f)
    A = a / (1 + n) * (1 + n ** 2 / 4 + n ** 4 / 64 + n ** 6 / 256)
    al = [n / 2 - 2 * n ** 2 / 3 + 5 * n ** 3 / 16 + 41 * n ** 4 / 180 - 127 * n ** 5 / 288 + 7891 * n ** 6 / 37800,
          13 * n ** 2 / 48 - 3 * n ** 3 / 5 + 557 * n ** 4 / 1440 + 281 * n ** 5 / 630 - 1983433 * n ** 6 / 1935360,
          61 * n ** 3 / 240 - 103 * n ** 4 / 140 + 15061 * n ** 5 / 26880 + 167603 * n ** 6 / 181440,
          49561 * n ** 4 / 161280 - 179 * n ** 5 / 168 + 6601661 * n ** 6 / 7257600,
          34729 * n ** 5 / 80640 - 3418889 * n ** 6 / 1995840,
          212378941 * n ** 6 / 319334400]
    phi = np.radians(lat)
    lam = np.radians(lon - (6.0 * zone - 183.0))
    c = 2 * math.sqrt(n) / (1 + n)
    t = np.sinh(np.arctanh(np.sin(phi)) - c * np.arctanh(c * np.sin(phi)))
    xi = np.arctan2(t, np.cos(lam))
    eta = np.arctanh(np.sin(lam) / np.sqrt(1 + t * t))
    se, sn = eta.copy(), xi.copy()
    for j in range(1, 7):
        se = se + al[j - 1] * np.cos(2 * j * xi) * np.sinh(2 * j * eta)
        sn = sn + al[j - 1] * np.sin(2 * j * xi) * np.cosh(2 * j * eta)
    return 500000.0 + k0 * A * se, (1e7 if south else 0.0) + k0 * A * sn


def dsm_grid(easts, norths, roi=None, resolution=0.5):
    """satellite_scene.py:524-538: (xoff, yoff, xsize, ysize, resolution)."""
    if roi is not None:
        xoff, yoff = float(roi[0]), float(roi[1])
        xsize = ysize = int(roi[2])
        resolution = float(roi[3])
        yoff += ysize * resolution
    else:
        xmin, xmax = float(np.min(easts)), float(np.max(easts))
        ymin, ymax = float(np.min(norths)), float(np.max(norths))
        xoff = np.floor(xmin / resolution) * resolution
        xsize = int(1 + np.floor((xmax - xoff) / resolution))
        yoff = np.ceil(ymax / resolution) * resolution
        ysize = int(1 - np.floor((ymin - yoff) / resolution))
    return xoff, yoff, xsize, ysize, resolution


def rasterize(cloud, xoff, yoff, resolution, xsize, ysize, radius=1, sigma=float("inf")):
    """plyflatten restated (see the header): (ysize, xsize) float64, NaN where empty."""
    cloud = np.asarray(cloud, np.float64)
    xx = (cloud[:, 0] - xoff) / resolution
    yy = (yoff - cloud[:, 1]) / resolution
    v = cloud[:, 2]
    ok = np.isfinite(xx) & np.isfinite(yy) & np.isfinite(v)
    xx, yy, v = xx[ok], yy[ok], v[ok]
    ci, cj = np.floor(xx).astype(np.int64), np.floor(yy).astype(np.int64)
    s = np.zeros(ysize * xsize)
    w = np.zeros(ysize * xsize)
    for dj in range(-radius, radius + 1):
        for di in range(-radius, radius + 1):
            ii, jj = ci + di, cj + dj
            m = (ii >= 0) & (jj >= 0) & (ii < xsize) & (jj < ysize)
            if math.isinf(sigma):
                wt = np.ones(int(m.sum()))
            else:
                d2 = (xx[m] - (ii[m] + 0.5)) ** 2 + (yy[m] - (jj[m] + 0.5)) ** 2
                wt = np.exp(-d2 / (2 * sigma * sigma))
            k = jj[m] * xsize + ii[m]
            np.add.at(s, k, wt * v[m])
            np.add.at(w, k, wt)
    out = np.full(ysize * xsize, np.nan)
    nz = w > 0
    out[nz] = s[nz] / w[nz]
    return out.reshape(ysize, xsize)


def dsm_mae(pred, gt):
    """modules/utils.py:142-245 on arrays, along its no-dsmr path (fix_xy: registration by the
    mean Z offset only, :197-201): MAE = nanmean |pred + nanmean(gt - pred) - gt|."""
    pred = np.asarray(pred, np.float64)
    gt = np.asarray(gt, np.float64)
    rp = pred + np.nanmean(gt - pred)
    return float(np.nanmean(np.abs(rp - gt)))
