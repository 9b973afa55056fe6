"""RPC ray generator.

CPU: the numpy restatement (oracle/rpc_ref.py) against rays produced by the reference's own
get_rays / normalize_rays / get_sun_dirs (tests/golden/rpc_rays.npz), and the localization
round trip that pins the rpcm restatement (rpcm itself: parity unpinned, not available).
GPU: spnerf_rpc_rays against the same fixture."""
import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import rpc_ref


def fixture():
    with np.load(f"{gu.GOLDEN}/rpc_rays.npz") as z:
        return {k: z[k] for k in z.files}


def rpc_from(arr, ds):
    d = dict(zip(rpc_ref.KEYS, arr[:10]))
    d.update(row_num=arr[10:30], row_den=arr[30:50], col_num=arr[50:70], col_den=arr[70:90])
    return rpc_ref.RPC(d, ds)


def pixels(meta):
    h, w, ds, lo, hi, r0, c0, nr, nc = meta
    rows, cols = np.meshgrid(np.arange(int(r0), int(r0 + nr)), np.arange(int(c0), int(c0 + nc)), indexing="ij")
    return cols.reshape(-1), rows.reshape(-1)


@pytest.mark.parametrize("tag", ["006_crop", "007_ds8"])
def test_oracle_rays_match_reference(tag):
    f = fixture()
    meta = f[f"{tag}|meta"]
    rpc = rpc_from(f[f"{tag}|rpc"], meta[2])
    cols, rows = pixels(meta)
    if tag == "007_ds8":   # keep the CPU test short: every 7th pixel
        cols, rows = cols[::7], rows[::7]
    rays = rpc_ref.get_rays(cols, rows, rpc, meta[3], meta[4])
    rays = rpc_ref.normalize_rays(rays, f["center"], f["range"])
    sun = rpc_ref.sun_dirs(*f[f"{tag}|sun_deg"], rays.shape[0])
    got = np.hstack([rays, sun])
    ref = f[f"{tag}|rays"][::7] if tag == "007_ds8" else f[f"{tag}|rays"]
    assert np.array_equal(got, ref)


def test_localization_round_trip():
    f = fixture()
    rpc = rpc_from(f["006_crop|rpc"], 1.0)
    rng = np.random.default_rng(0)
    cols, rows = rng.uniform(0, 793, 500), rng.uniform(0, 813, 500)
    for alt in (-30.0, -2.0, 15.0):
        lon, lat = rpc.localization(cols, rows, np.full(500, alt))
        c2, r2 = rpc.projection(lon, lat, alt)
        assert np.abs(c2 - cols).max() < 1e-6 and np.abs(r2 - rows).max() < 1e-6


def test_sun_direction_formula():
    f = fixture()
    np.testing.assert_array_equal(rpc_ref.sun_dirs(60.0, 140.0, 2), f["sun_60_140"])


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["006_crop", "007_ds8"])
def test_gpu_rays_match_reference(tag):
    from spnerf_amd import satellite
    f = fixture()
    meta = f[f"{tag}|meta"]
    h, w, ds, lo, hi, r0, c0, nr, nc = meta
    cams = satellite.load_cameras()
    name = {"006_crop": "JAX_269_006_RGB", "007_ds8": "JAX_269_007_RGB"}[tag]
    got = satellite.image_rays(cams["images"][name], ds, cams["scene_loc"], crop=(int(r0), int(c0), int(nr), int(nc)))
    ref = f[f"{tag}|rays"]
    got = got.cpu().numpy()
    # directions, near/far and sun to fp32 rounding; origins are ECEF rounded to fp32 (0.5 m) before
    # centring, so a last-bit difference of the fp64 ECEF may flip at most a handful of them by one quantum
    np.testing.assert_allclose(got[:, 3:], ref[:, 3:], rtol=0, atol=2e-7)
    diff = np.abs(got[:, :3] - ref[:, :3])
    quantum = 0.5 / float(f["range"])
    assert diff.max() <= quantum * 1.01
    assert (diff > 0).sum() <= max(2, ref.shape[0] // 2000), (diff > 0).sum()


@pytest.mark.gpu
def test_gpu_get_rays_pixel_list_matches_oracle():
    from spnerf_amd import satellite
    cams = satellite.load_cameras()
    meta = cams["images"]["JAX_269_011_RGB"]
    rng = np.random.default_rng(1)
    cols, rows = rng.integers(0, meta["width"], 300), rng.integers(0, meta["height"], 300)
    rpc = satellite.RPCModel(meta["rpc"])
    got = satellite.get_rays(cols, rows, rpc, meta["min_alt"], meta["max_alt"]).cpu().numpy()
    ref = rpc_ref.get_rays(cols.astype(float), rows.astype(float), rpc_ref.RPC(meta["rpc"]), meta["min_alt"],
                           meta["max_alt"])
    np.testing.assert_allclose(got[:, 3:], ref[:, 3:], rtol=1e-6, atol=1e-7)
    assert np.abs(got[:, :3] - ref[:, :3]).max() <= 1.0   # ECEF metres: at most one fp32 quantum (0.5 m)
