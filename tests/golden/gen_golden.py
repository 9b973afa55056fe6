"""Generate the golden fixtures by running the REFERENCE render path in this container.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [--ref /root/reference]

Only this script reads ``/root/reference``; it runs here (the build container),
never on the GPU box.  It imports the reference's ``models/spnerf.py`` and
``modules/rendering.py`` (pure torch/numpy), records every
random tensor the reference draws (``torch.rand``/``rand_like``/``randn``
are wrapped, not replaced), and stores inputs, recorded randoms, outputs and
gradients as small ``.npz`` files next to this script.  Weights are NOT
stored: they are rebuilt from ``oracle/weights.make_weights(dims, seed)``.

Gradients are taken of a fixed random-projection loss
``L = Σ_k <out_k, R_k>`` over every differentiable output ``k`` of
``render_rays`` (``R_k`` drawn from ``numpy.random.default_rng(1234)`` in
sorted key order, see ``projection_weights``), which exercises the backward
of every returned tensor.  For W=512 the full gradients would be too large,
so those cases store per-parameter projections ``<∂L/∂θ, Q_θ>`` instead.
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.weights import ModelDims, make_weights  # noqa: E402


# helpers shared with the tests live in tests/golden_util.py (the GPU tests never load this file)
sys.path.insert(0, os.path.dirname(HERE))
from golden_util import param_projections, projection_weights, synthetic_rays  # noqa: E402


# ------------------------------------------------------------------ reference driver

class Recorder:
    """Wraps torch's RNG entry points used by the reference and records outputs."""

    def __init__(self):
        self.draws = []
        self._orig = {}

    def __enter__(self):
        for name in ("rand", "rand_like", "randn"):
            fn = getattr(torch, name)
            self._orig[name] = fn

            def wrapped(*a, __fn=fn, __name=name, **kw):
                t = __fn(*a, **kw)
                self.draws.append(("randn" if __name == "randn" else "rand", t.detach().clone()))
                return t
            setattr(torch, name, wrapped)
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            setattr(torch, name, fn)


def load_reference(ref: str):
    sys.path.insert(0, ref)
    sys.dont_write_bytecode = True
    import models.spnerf as ref_spnerf  # noqa
    import modules.rendering as ref_rendering  # noqa
    return ref_spnerf, ref_rendering


def build_model(ref_spnerf, dims: ModelDims, seed: int):
    m = ref_spnerf.SPNeRF(num_sem_classes=dims.num_sem_classes, s_embedding_factor=dims.s_embedding_factor,
                          layers=dims.layers, feat=dims.width, mapping=dims.mapping, t_embedding_dims=dims.t_dim,
                          beta=dims.beta, sem=dims.sem)
    w = make_weights(dims, seed)
    sd = m.state_dict()
    assert list(sd.keys()) == list(w.keys()), (list(sd.keys()), list(w.keys()))
    m.load_state_dict({k: torch.tensor(v) for k, v in w.items()})
    return m


def make_args(**kw):
    base = dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=False, sc_lambda=0.0,
                margin=0.0001, stdscale=1.0, chunk=5120, noise_std=0.0)
    base.update(kw)
    return types.SimpleNamespace(**base)


def run_case(ref_spnerf, ref_rendering, name: str, dims: ModelDims, args, n_rays: int, mode: str,
             full_grads: bool, seed: int = 0, with_depth: bool = False, torch_seed: int = 0,
             t_vocab: int = 30, rays_np=None):
    torch.manual_seed(torch_seed)
    model = build_model(ref_spnerf, dims, seed)
    models = {"coarse": model}
    if args.n_importance > 0:   # second network, weights from seed + 100
        models["fine"] = build_model(ref_spnerf, dims, seed + 100)
    rays = torch.tensor(synthetic_rays(n_rays, seed=100 + seed) if rays_np is None else rays_np[:n_rays])
    rng = np.random.default_rng(7 + seed)
    sem = ts = None
    extra = {}
    if dims.sem:
        labels = rng.choice([0, 1, 2, -100], size=n_rays, p=[0.35, 0.3, 0.25, 0.10]).astype(np.int64)
        labels[labels >= dims.num_sem_classes] = -100
        sem = torch.tensor(labels)
        extra["semantics"] = labels
    if dims.beta:
        emb_t = torch.nn.Embedding(t_vocab, dims.t_dim)
        with torch.no_grad():
            emb_t.weight.copy_(torch.tensor(np.random.default_rng(99).standard_normal((t_vocab, dims.t_dim)).astype(np.float32)))
        models["t"] = emb_t
        ts_np = rng.integers(0, t_vocab, size=n_rays).astype(np.int64)
        ts = torch.tensor(ts_np)
        extra["ts"] = ts_np
        extra["t_embedding"] = emb_t.weight.detach().numpy().copy()
    kw = {}
    if with_depth:
        valid = (rng.uniform(size=n_rays) < 0.68).astype(np.int64)
        far = rays[:, 7].numpy()
        gt = (far * rng.uniform(0.3, 0.7, size=n_rays)).astype(np.float32)
        corr = rng.uniform(0.2, 1.0, size=n_rays).astype(np.float32)
        std = ((1.0 - rng.uniform(0, 1, size=n_rays)) * 0.05 + 1e-4).astype(np.float32)
        kw = dict(valid_depth=torch.tensor(valid), target_depths=torch.tensor(np.stack([gt, corr], 1)),
                  target_std=torch.tensor(std))
        extra.update(valid_depth=valid, target_depths=np.stack([gt, corr], 1), target_std=std)
    with Recorder() as rec:
        res = ref_rendering.render_rays(models, args, rays, ts, semantics=sem, mode=mode, **kw)
    outs = {k: v for k, v in res.items() if torch.is_tensor(v)}
    shapes = {k: tuple(v.shape) for k, v in outs.items() if v.requires_grad}
    R = projection_weights(shapes)
    loss = sum((outs[k] * torch.tensor(R[k])).sum() for k in sorted(R))
    params = list(model.named_parameters())
    if "fine" in models:
        params += [("fine." + n, p) for n, p in models["fine"].named_parameters()]
    if dims.beta:
        params += [("t.weight", models["t"].weight)]
    loss.backward()
    data = {"rays": rays.numpy()}
    for k, v in extra.items():
        data["in_" + k] = v
    for i, (kind, t) in enumerate(rec.draws):
        data[f"rng{i:02d}_{kind}"] = t.numpy()
    for k, v in outs.items():
        data["out_" + k] = v.detach().numpy()
    if full_grads:
        for n, p in params:   # a parameter the outputs do not depend on has no .grad → zeros
            data["grad_" + n] = p.grad.numpy() if p.grad is not None else np.zeros(tuple(p.shape), np.float32)
    else:
        Q = param_projections([(n, tuple(p.shape)) for n, p in params])
        for n, p in params:
            data["gproj_" + n] = np.array((p.grad.double() * torch.tensor(Q[n]).double()).sum().item())
            data["gnorm_" + n] = np.array(p.grad.double().norm().item())
    data["loss"] = np.array(loss.item())
    meta = dict(dims=dims.__dict__, args=args.__dict__, mode=mode, seed=seed, n_rays=n_rays)
    data["meta"] = np.array(repr(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **data)
    print(f"{name}: {len(rec.draws)} draws, {os.path.getsize(path) / 1e3:.1f} kB")


def unit_sampling(ref_rendering):
    """sample_pdf / sample_3sigma on edge-case windows (clamped, tiny std, wide)."""
    torch.manual_seed(5)
    B, N = 48, 64
    rng = np.random.default_rng(11)
    depth = rng.uniform(0.0, 0.25, size=B).astype(np.float32)
    std = np.concatenate([rng.uniform(1e-4, 2e-3, 16), rng.uniform(0.01, 0.05, 16), rng.uniform(0.1, 0.5, 16)]).astype(np.float32)
    low, high = torch.tensor(depth - 3 * std), torch.tensor(depth + 3 * std)
    near, far = torch.tensor(0.0), torch.tensor(0.21)
    with Recorder() as rec:
        s3 = ref_rendering.sample_3sigma(low, high, N, False, near, far)
    bins = torch.sort(torch.rand(B, 33), -1)[0]
    w = torch.rand(B, 32) ** 4
    w[:4] = 0.0
    with Recorder() as rec2:
        sp = ref_rendering.sample_pdf(bins, w, 40, det=False)
    # NOTE: det=True raises in the reference (1-D linspace u vs (B, S_+1) cdf in
    # torch.searchsorted, rendering.py:33,38); perturb is hard-coded to 1 so it never runs.
    np.savez_compressed(os.path.join(HERE, "unit_sampling.npz"), low=low.numpy(), high=high.numpy(), near=0.0, far=0.21,
                        u3=rec.draws[0][1].numpy(), s3=s3.numpy(), bins=bins.numpy(), w=w.numpy(),
                        u_pdf=rec2.draws[0][1].numpy(), s_pdf=sp.numpy())
    print("unit_sampling written")


def unit_composite(ref_spnerf):
    """inference() compositing driven by a stub model returning chosen raw outputs, covering
    opaque (σ≫1), empty (σ≈0) and mixed rays; full gradients w.r.t. the raw outputs."""
    B, S, C = 40, 64, 3
    rng = np.random.default_rng(21)
    raw = rng.uniform(0, 1, size=(B, S, 8 + C)).astype(np.float32)
    sig = rng.exponential(2.0, size=(B, S)).astype(np.float32)
    sig[:8] *= 1e3        # opaque
    sig[8:16] *= 1e-6     # empty
    sig[16:20] = 0.0
    raw[..., 3] = sig
    raw[..., 8:] = rng.standard_normal((B, S, C))
    z = np.sort(rng.uniform(0, 0.2, size=(B, S)).astype(np.float32), -1)
    raw_t = torch.tensor(raw.reshape(B * S, -1), requires_grad=True)

    class Stub(torch.nn.Module):
        number_of_outputs, beta, sem = 8 + C, False, True

        def forward(self, x, **kw):
            return raw_t[: x.shape[0]]

    args = make_args(chunk=B * S, noise_std=0.3)
    torch.manual_seed(3)
    with Recorder() as rec:
        res = ref_spnerf.inference(Stub(), args, torch.zeros(B, S, 3), torch.tensor(z),
                                   sun_d=torch.zeros(B, 3))
    shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
    R = projection_weights(shapes)
    sum((res[k] * torch.tensor(R[k])).sum() for k in sorted(R)).backward()
    np.savez_compressed(os.path.join(HERE, "unit_composite.npz"), raw=raw, z=z, noise=rec.draws[0][1].numpy(),
                        noise_std=0.3, **{"out_" + k: v.detach().numpy() for k, v in res.items()},
                        grad_raw=raw_t.grad.numpy())
    print("unit_composite written")


def dropins(ref_spnerf, ref_rendering):
    """The public drop-ins outside render_rays, through the reference itself:
    inference() on explicit sample positions (spnerf.py:63-159, noise on, sem on),
    compute_samples_around_depth (rendering.py:76-89) and GenerateGuidedSamples in test and
    train mode (:92-116; its output is in DRAW order, render_rays sorts afterwards at :165),
    and load_model(args) (models/__init__.py:4-16) after torch.manual_seed(9)."""
    from models import load_model
    dims = ModelDims(width=64, sem=True)
    torch.manual_seed(0)
    model = build_model(ref_spnerf, dims, 12)
    B, S = 24, 32
    rays = torch.tensor(synthetic_rays(B, seed=120))
    rng = np.random.default_rng(13)
    far = rays[:, 7:8]
    z = torch.tensor(np.sort(rng.uniform(0, 1, (B, S)), -1).astype(np.float32)) * far
    xyz = rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]
    sem = torch.tensor(rng.choice([0, 1, 2, -100], size=B).astype(np.int64))
    args = make_args(n_samples=S, noise_std=0.2)
    with Recorder() as rec:
        res = ref_spnerf.inference(model, args, xyz, z, sun_d=rays[:, 8:11], semantics=sem)
    outs = {k: v for k, v in res.items() if torch.is_tensor(v)}
    R = projection_weights({k: tuple(v.shape) for k, v in outs.items() if v.requires_grad})
    sum((outs[k] * torch.tensor(R[k])).sum() for k in sorted(R)).backward()
    data = {"rays": rays.numpy(), "z": z.numpy(), "xyz": xyz.numpy(), "in_semantics": sem.numpy(),
            "noise_std": np.array(0.2), "rng00_randn": rec.draws[0][1].numpy()}
    data.update({"out_" + k: v.detach().numpy() for k, v in outs.items()})
    data.update({"grad_" + n: p.grad.numpy() for n, p in model.named_parameters()})
    # guided sampling around the rendered depth, clamped to the first ray's [near, far]
    rd = {"depth": res["depth"].detach(), "weights": res["weights"].detach()}
    near, far2 = rays[:, 6:7], rays[:, 7:8]
    with Recorder() as rc:
        zc = ref_rendering.compute_samples_around_depth(rd, S, z, 1.0, near[0, 0], far2[0, 0])
    data.update(csad_u=rc.draws[0][1].numpy(), csad_out=zc.numpy())
    with Recorder() as rt:
        zt = ref_rendering.GenerateGuidedSamples(rd, z, S, 1.0, near, far2, mode="test")
    data.update(ggs_test_u=rt.draws[0][1].numpy(), ggs_test_out=zt.numpy())
    valid = (rng.uniform(size=B) < 0.6).astype(np.int64)
    td = np.stack([(far[:, 0].numpy() * rng.uniform(0.3, 0.7, B)), rng.uniform(0.2, 1, B)], 1).astype(np.float32)
    tstd = ((1 - rng.uniform(0, 1, B)) * 0.05 + 1e-4).astype(np.float32)
    with Recorder() as rr:
        ztr = ref_rendering.GenerateGuidedSamples(rd, z, S, 1.0, near, far2, mode="train", valid_depth=torch.tensor(valid),
                                                  target_depths=torch.tensor(td), target_std=torch.tensor(tstd))
    data.update(ggs_train_u0=rr.draws[0][1].numpy(), ggs_train_u1=rr.draws[1][1].numpy(), ggs_train_out=ztr.numpy(),
                in_valid_depth=valid, in_target_depths=td, in_target_std=tstd)
    # load_model(args): the reference's factory and initialisation
    margs = types.SimpleNamespace(model="sp-nerf", num_sem_classes=3, s_embedding_factor=1, fc_layers=8, fc_units=64,
                                  mapping=True, t_embbeding_tau=4, beta=True, sem=True)
    torch.manual_seed(9)
    lm = load_model(margs)
    Q = param_projections([(n, tuple(p.shape)) for n, p in lm.named_parameters()])
    for n, p in lm.named_parameters():
        data[f"load_model|{n}|sum"] = np.array(p.detach().double().sum().item())
        data[f"load_model|{n}|proj"] = np.array((p.detach().double() * torch.tensor(Q[n]).double()).sum().item())
    data["load_model|number_of_outputs"] = np.array(lm.number_of_outputs)
    np.savez_compressed(os.path.join(HERE, "dropins_w64.npz"), **data)
    print("dropins_w64 written")


def load_metrics(ref: str):
    """modules/metrics.py with its only non-torch import (kornia, for SSIM) stubbed."""
    from unittest import mock
    saved = {k: sys.modules.get(k) for k in ("kornia", "kornia.losses")}
    for k in saved:
        sys.modules[k] = mock.MagicMock()
    try:
        import modules.metrics as metrics
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return metrics


def losses(ref: str):
    """The reference losses (modules/metrics.py:10-207) on render-shaped random inputs: SNerfLoss
    (+ solar terms, + fine keys), SatNerfLoss (β uncertainty), DepthLoss in its subset MSE, subset
    GNLL and use-all-depth forms, SemanticLoss (ignore_index -100, + fine), psnr.  Stores the
    inputs, every loss value and the gradient w.r.t. every differentiable input."""
    metrics = load_metrics(ref)
    rng = np.random.default_rng(31)
    B, S, C = 40, 24, 3
    t = lambda a: torch.tensor(np.asarray(a, np.float32), requires_grad=True)
    data = {}
    inp = {}
    for typ in ("coarse", "fine"):
        w = rng.uniform(0, 1, (B, S)) ** 3
        w = w / w.sum(1, keepdims=True) * rng.uniform(0.6, 1.0, (B, 1))
        z = np.sort(rng.uniform(0, 0.2, (B, S)), 1)
        raw = dict(rgb=rng.uniform(0, 1, (B, 3)), depth=(w * z).sum(1), weights=w, z_vals=z,
                   sun_sc=rng.uniform(0, 1, (B, S, 1)), transparency_sc=np.cumprod(rng.uniform(0.8, 1, (B, S)), 1),
                   weights_sc=rng.uniform(0, 0.1, (B, S)), sem_logits=rng.normal(size=(B, C)),
                   beta=rng.uniform(0.01, 0.5, (B, S, 1)))
        for k, v in raw.items():
            inp[f"{k}_{typ}"] = v.astype(np.float32)
    targets = rng.uniform(0, 1, (B, 3)).astype(np.float32)
    depth_t = (inp["depth_coarse"] * rng.uniform(0.7, 1.3, B)).astype(np.float32)
    depth_w = rng.uniform(0.2, 1, B).astype(np.float32)
    valid = (rng.uniform(size=B) < 0.7).astype(np.int64)
    dstd = rng.uniform(1e-3, 0.02, B).astype(np.float32)
    labels = rng.choice([0, 1, 2, -100], size=B, p=[0.3, 0.3, 0.25, 0.15]).astype(np.int64)
    data.update({"in_" + k: v for k, v in inp.items()})
    data.update(in_targets=targets, in_depth_t=depth_t, in_depth_w=depth_w, in_valid=valid, in_dstd=dstd,
                in_labels=labels)

    def run(tag, keys, fn):
        tens = {k: t(inp[k]) for k in keys}
        loss, ld = fn(tens)
        loss.backward()
        data[f"{tag}|loss"] = np.array(float(loss))
        for k, v in ld.items():
            data[f"{tag}|term|{k}"] = np.array(float(v))
        for k, v in tens.items():
            data[f"{tag}|grad|{k}"] = (v.grad if v.grad is not None else torch.zeros_like(v)).numpy()

    co = [k for k in inp if k.endswith("_coarse")]
    al = list(inp)
    tg = torch.tensor(targets)
    dt, dw, dv, ds = torch.tensor(depth_t), torch.tensor(depth_w), torch.tensor(valid), torch.tensor(dstd)
    run("snerf_sc", co, lambda x: metrics.SNerfLoss(lambda_sc=0.1)(x, tg))
    run("snerf_fine", al, lambda x: metrics.SNerfLoss(lambda_sc=0.05)(x, tg))
    run("satnerf_sc", co, lambda x: metrics.SatNerfLoss(lambda_sc=0.1)(x, tg))
    run("satnerf_fine", al, lambda x: metrics.SatNerfLoss(lambda_sc=0.0)(x, tg))
    run("depth_subset", co, lambda x: metrics.DepthLoss(lambda_ds=1.0, usealldepth=False)(x, dt, dw, dv, ds))
    run("depth_subset_fine", al, lambda x: metrics.DepthLoss(lambda_ds=0.7, usealldepth=False)(x, dt, dw, dv, ds))
    run("depth_gnll", co, lambda x: metrics.DepthLoss(lambda_ds=1.0, GNLL=True, usealldepth=False)(x, dt, dw, dv, ds))
    run("depth_all", al, lambda x: metrics.DepthLoss(lambda_ds=1.0, usealldepth=True)(x, dt, dw, dv, ds))
    lab = torch.tensor(labels)
    run("sem", co, lambda x: metrics.SemanticLoss(lambda_ss=0.04)(x, lab))
    run("sem_fine", al, lambda x: metrics.SemanticLoss(lambda_ss=1.0)(x, lab))
    data["psnr"] = np.array(float(metrics.psnr(torch.tensor(inp["rgb_coarse"]), tg)))
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **data)
    print("losses written", len(data), "arrays")


def init_weights(ref_spnerf):
    """SPNeRF(...) built after torch.manual_seed(7): the reference's own initialisation, for the
    seeded-init equivalence test of the drop-in module (stored as per-parameter sums and
    projections, not the weights)."""
    out = {}
    for tag, kw in (("w64_sem_beta", dict(num_sem_classes=3, feat=64, mapping=True, sem=True, beta=True,
                                          t_embedding_dims=4)),
                    ("w512", dict(feat=512, mapping=True))):
        torch.manual_seed(7)
        m = ref_spnerf.SPNeRF(**kw)
        Q = param_projections([(n, tuple(p.shape)) for n, p in m.named_parameters()])
        for n, p in m.named_parameters():
            out[f"{tag}|{n}|sum"] = np.array(p.detach().double().sum().item())
            out[f"{tag}|{n}|proj"] = np.array((p.detach().double() * torch.tensor(Q[n]).double()).sum().item())
    np.savez_compressed(os.path.join(HERE, "init_seed7.npz"), **out)
    print("init_seed7 written")


def rpc_rays(ref: str) -> dict:
    """Rays of JAX_269 views through the reference's own datasets/satellite_scene.py get_rays
    (:21-68, with modules/utils.py geodetic_to_ecef :80-100), normalize_rays (:415-425) and
    get_sun_dirs (:449-473).  Its I/O-only imports (rasterio, rpcm, torchvision, cv2, …) are
    replaced by MagicMock modules; the rpcm localization it calls is the numpy restatement
    oracle/rpc_ref.RPC (rpcm itself is unavailable offline and unpinned — SURVEY §8c)."""
    import json
    import types
    from unittest import mock
    from oracle.rpc_ref import RPC
    stubs = ["rasterio", "rpcm", "torchvision", "torchvision.transforms", "cv2", "pyproj", "utm", "osgeo", "gdal",
             "plyflatten", "kornia", "kornia.losses", "srtm4", "numba", "lpips", "PIL", "PIL.Image"]
    saved = {k: sys.modules.get(k) for k in stubs}
    for k in stubs:
        sys.modules[k] = mock.MagicMock()
    try:
        import datasets.satellite_scene as ss
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    jdir = os.path.join(ref, "Dataset", "DFC2019_269", "JSON")
    loc = json.load(open(os.path.join(jdir, "scene.loc")))
    center = torch.tensor([float(loc["X_offset"]), float(loc["Y_offset"]), float(loc["Z_offset"])])
    rng = torch.max(torch.tensor([float(loc["X_scale"]), float(loc["Y_scale"]), float(loc["Z_scale"])]))
    holder = types.SimpleNamespace(center=center, range=rng)
    out = {"center": center.numpy(), "range": np.array(rng.item(), np.float32)}
    for tag, img, ds, crop in (("006_crop", "JAX_269_006_RGB.json", 1.0, (400, 400, 16, 16)),
                               ("007_ds8", "JAX_269_007_RGB.json", 8.0, None)):
        d = json.load(open(os.path.join(jdir, img)))
        h, w = int(d["height"] // ds), int(d["width"] // ds)
        rpc = RPC(d["rpc"], ds)
        cols, rows = np.meshgrid(np.arange(w), np.arange(h))
        cols, rows = cols.flatten(), rows.flatten()
        if crop:
            r0, c0, ch, cw = crop
            sel = (rows >= r0) & (rows < r0 + ch) & (cols >= c0) & (cols < c0 + cw)
            cols, rows = cols[sel], rows[sel]
        rays = ss.get_rays(cols, rows, rpc, float(d["min_alt"]), float(d["max_alt"]))
        rays = ss.SatelliteSceneDataset.normalize_rays(holder, rays)
        sun = ss.SatelliteSceneDataset.get_sun_dirs(holder, float(d["sun_elevation"]), float(d["sun_azimuth"]),
                                                    rays.shape[0])
        out[f"{tag}|rays"] = torch.hstack([rays, sun]).numpy()
        out[f"{tag}|meta"] = np.array([h, w, ds, float(d["min_alt"]), float(d["max_alt"]),
                                       *(crop if crop else (0, 0, h, w))], np.float64)
        out[f"{tag}|rpc"] = np.array([d["rpc"][k] for k in ("row_offset", "col_offset", "lat_offset", "lon_offset",
                                      "alt_offset", "row_scale", "col_scale", "lat_scale", "lon_scale", "alt_scale")]
                                     + list(d["rpc"]["row_num"]) + list(d["rpc"]["row_den"])
                                     + list(d["rpc"]["col_num"]) + list(d["rpc"]["col_den"]), np.float64)
        out[f"{tag}|sun_deg"] = np.array([float(d["sun_elevation"]), float(d["sun_azimuth"])])
    # a non-trivial sun direction through the reference formula as well
    out["sun_60_140"] = ss.SatelliteSceneDataset.get_sun_dirs(holder, 60.0, 140.0, 2).numpy()
    np.savez_compressed(os.path.join(HERE, "rpc_rays.npz"), **out)
    print("rpc_rays written", {k: v.shape for k, v in out.items() if k.endswith("rays")})
    return out


def dsm_latlon(ref: str) -> None:
    """datasets/satellite_scene.py:475-505 (get_latlonalt_from_nerf_prediction, with
    modules/utils.py:103-122 ecef_to_latlon_custom) run by the reference itself on 4096 real
    JAX_269_007 rays (rpc_rays.npz, ds 8) at a drawn depth between each ray's near and far; its
    I/O-only imports stubbed as in rpc_rays.  Pins oracle/dsm_ref.latlonalt_from_prediction and
    spnerf_dsm_points.  (Its UTM step calls pyproj and the DSM step plyflatten: both absent, so
    those stay parity unpinned.)"""
    import json
    import types
    from unittest import mock
    stubs = ["rasterio", "rpcm", "torchvision", "torchvision.transforms", "cv2", "pyproj", "utm", "osgeo", "gdal",
             "plyflatten", "kornia", "kornia.losses", "srtm4", "numba", "lpips", "PIL", "PIL.Image"]
    saved = {k: sys.modules.get(k) for k in stubs}
    for k in stubs:
        sys.modules[k] = mock.MagicMock()
    try:
        import datasets.satellite_scene as ss
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    jdir = os.path.join(ref, "Dataset", "DFC2019_269", "JSON")
    loc = json.load(open(os.path.join(jdir, "scene.loc")))
    center = torch.tensor([float(loc["X_offset"]), float(loc["Y_offset"]), float(loc["Z_offset"])])
    rng = torch.max(torch.tensor([float(loc["X_scale"]), float(loc["Y_scale"]), float(loc["Z_scale"])]))
    holder = types.SimpleNamespace(center=center, range=rng)
    rays_all = np.load(os.path.join(HERE, "rpc_rays.npz"))["007_ds8|rays"]
    sel = np.sort(np.random.default_rng(0).choice(rays_all.shape[0], 4096, replace=False))
    rays = torch.tensor(rays_all[sel])
    g = torch.Generator().manual_seed(0)
    depth = rays[:, 6] + (rays[:, 7] - rays[:, 6]) * torch.rand(rays.shape[0], generator=g)
    lats, lons, alts = ss.SatelliteSceneDataset.get_latlonalt_from_nerf_prediction(holder, rays, depth.view(-1, 1))
    np.savez_compressed(os.path.join(HERE, "dsm_latlon.npz"), rays=rays.numpy(), depth=depth.numpy(),
                        center=center.numpy(), range=np.array(rng.item(), np.float32), lats=np.asarray(lats),
                        lons=np.asarray(lons), alts=np.asarray(alts))
    print("dsm_latlon written", rays.shape)
    # DSM end-to-end data: every JAX_269_007 ds-8 ray with the depth at which it meets the lidar
    # ground truth (Truth/JAX_269_DSM.tif on its ROI grid, Truth/JAX_269_DSM.txt), found by
    # bisection through the oracle's lat/lon/alt + UTM (geometry input only — the expected
    # values are the reference's lidar DSM itself, stored as float16 heights: 1.6 cm steps)
    from PIL import Image
    from oracle import dsm_ref
    tdir = os.path.join(ref, "Dataset", "DFC2019_269", "Truth")
    gt = np.array(Image.open(os.path.join(tdir, "JAX_269_DSM.tif")), np.float64)
    roi = np.loadtxt(os.path.join(tdir, "JAX_269_DSM.txt"))
    xoff, yoff, xsize, ysize, res = dsm_ref.dsm_grid(None, None, roi=roi)
    r = rays_all.astype(np.float64)
    c = center.numpy().astype(np.float64)
    rg = float(np.float32(rng.item()))
    lat0, lon0, _ = dsm_ref.latlonalt_from_prediction(r[:1], r[:1, 6], c, rg)
    zone = dsm_ref.utm_zone(float(lat0[0]), float(lon0[0]))[0]

    def f(t):
        la, lo, al = dsm_ref.latlonalt_from_prediction(r, t, c, rg)
        e, n = dsm_ref.utm(la, lo, zone)
        i = np.floor((e - xoff) / res).astype(np.int64)
        j = np.floor((yoff - n) / res).astype(np.int64)
        ok = (i >= 0) & (j >= 0) & (i < xsize) & (j < ysize)
        h = np.full(t.shape, np.nan)
        h[ok] = gt[j[ok], i[ok]]
        return al - h

    lo_t, hi_t = r[:, 6].copy(), r[:, 7].copy()
    for _ in range(60):
        mid = 0.5 * (lo_t + hi_t)
        fm = f(mid)
        above = fm > 0   # the ray is still above the surface: go deeper
        lo_t = np.where(above, mid, lo_t)
        hi_t = np.where(above, hi_t, mid)
    t = 0.5 * (lo_t + hi_t)
    hit = np.isfinite(f(t))
    np.savez_compressed(os.path.join(HERE, "dsm_truth.npz"), rays=rays_all[hit], depth=t[hit].astype(np.float32),
                        center=center.numpy(), range=np.array(rng.item(), np.float32), roi=roi,
                        gt=gt.astype(np.float16), zone=np.array(zone))
    print("dsm_truth written", int(hit.sum()), "of", r.shape[0], "rays on the ROI")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="regenerate one fixture group only (dsm)")
    a = ap.parse_args()
    torch.set_num_threads(8)
    if a.only == "dsm":
        sys.path.insert(0, a.ref)
        sys.dont_write_bytecode = True
        dsm_latlon(a.ref)
        return
    ref_spnerf, ref_rendering = load_reference(a.ref)
    real = rpc_rays(a.ref)
    # config 1: the 16x16 crop of JAX_269_006 (rows/cols 400-415; rays through the reference's
    # get_rays / normalize_rays / get_sun_dirs), 256 rays x 64 samples, coarse, mapping, W=512
    run_case(ref_spnerf, ref_rendering, "c1_w512", ModelDims(width=512), make_args(), 256, "test", full_grads=False,
             rays_np=real["006_crop|rays"])
    # small full-gradient case of the same path
    run_case(ref_spnerf, ref_rendering, "c1_w64", ModelDims(width=64), make_args(), 64, "train", full_grads=True, seed=1)
    # README recipe path (config 3 flags): guided + solar correction + semantics, train mode with depth priors
    c3 = make_args(guidedsample=True, sc_lambda=0.1)
    run_case(ref_spnerf, ref_rendering, "c3_w64", ModelDims(width=64, sem=True), c3, 64, "train",
             full_grads=True, seed=2, with_depth=True)
    run_case(ref_spnerf, ref_rendering, "c3_w512", ModelDims(width=512, sem=True), c3, 48, "train",
             full_grads=False, seed=3, with_depth=True)
    run_case(ref_spnerf, ref_rendering, "c3_test_w64", ModelDims(width=64, sem=True), c3, 32, "test",
             full_grads=True, seed=4)
    # beta head + time embedding, noise on
    run_case(ref_spnerf, ref_rendering, "beta_w64", ModelDims(width=64, sem=True, beta=True),
             make_args(beta=True, sc_lambda=0.05, noise_std=0.5), 32, "train", full_grads=True, seed=5)
    # hierarchical fine model (rendering.py:186-216): plain, and with the solar pass (which in the
    # reference replaces the coarse dictionary by the fine solar inference's, :207)
    run_case(ref_spnerf, ref_rendering, "fine_w64", ModelDims(width=64, sem=True), make_args(n_importance=32),
             32, "test", full_grads=True, seed=7)
    run_case(ref_spnerf, ref_rendering, "fine_sc_guided_w64", ModelDims(width=64),
             make_args(n_importance=48, sc_lambda=0.1, guidedsample=True), 24, "train", full_grads=True, seed=8,
             with_depth=True)
    # no positional encoding (mapping off), n_samples=32
    run_case(ref_spnerf, ref_rendering, "nomap_w64", ModelDims(width=64, mapping=False),
             make_args(n_samples=32), 40, "test", full_grads=True, seed=6)
    # config 5 flags: 128 stratified samples/ray, semantic head on (C=3), W=512, test mode
    run_case(ref_spnerf, ref_rendering, "c5_w512", ModelDims(width=512, sem=True), make_args(n_samples=128), 64, "test",
             full_grads=False, seed=10)
    unit_sampling(ref_rendering)
    unit_composite(ref_spnerf)
    init_weights(ref_spnerf)
    dropins(ref_spnerf, ref_rendering)
    losses(a.ref)
    dsm_latlon(a.ref)


if __name__ == "__main__":
    main()
