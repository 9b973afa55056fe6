"""The CPU oracle (oracle/ref_cpu.py) against fixtures produced by the REFERENCE itself
(tests/golden/gen_golden.py): pins the oracle before it is trusted as a checker."""
import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import ref_cpu
from oracle.weights import make_weights


def run_oracle(name):
    data = gu.load(name)
    meta = data["meta"]
    dims, args = gu.dims_of(meta), gu.args_of(meta)
    p = ref_cpu.to_params(make_weights(dims, meta["seed"]), requires_grad=True)
    pf = ref_cpu.to_params(make_weights(dims, meta["seed"] + 100), requires_grad=True) if args.n_importance else None
    replay = gu.Replay(gu.draws_of(data), torch.tensor)
    rays = torch.tensor(data["rays"])
    sem = torch.tensor(data["in_semantics"]) if "in_semantics" in data else None
    ts = torch.tensor(data["in_ts"]) if "in_ts" in data else None
    emb_t = torch.tensor(data["in_t_embedding"], requires_grad=True) if "in_t_embedding" in data else None
    kw = {}
    if "in_valid_depth" in data:
        kw = dict(valid_depth=torch.tensor(data["in_valid_depth"]), target_depths=torch.tensor(data["in_target_depths"]),
                  target_std=torch.tensor(data["in_target_std"]))
    res = ref_cpu.render_rays(p, dims, args, rays, ts, sem, meta["mode"], t_embed=(lambda t: emb_t[t]) if emb_t is not None else None,
                              draw=replay, fine_params=pf, **kw)
    assert replay.used == len(replay.draws)
    if pf is not None:
        p = dict(p, **{"fine." + k: v for k, v in pf.items()})
    return data, p, emb_t, res


@pytest.mark.parametrize("name", gu.CASES)
def test_oracle_outputs_match_reference(name):
    data, p, emb_t, res = run_oracle(name)
    keys = sorted(k[4:] for k in data if k.startswith("out_"))
    assert sorted(res.keys()) == keys
    for k in keys:
        gu.assert_close(k, res[k].detach().numpy(), data["out_" + k], rtol=2e-5, atol_frac=1e-6)


@pytest.mark.parametrize("name", gu.CASES)
def test_oracle_grads_match_reference(name):
    data, p, emb_t, res = run_oracle(name)
    shapes = {k: tuple(v.shape) for k, v in res.items() if v.requires_grad}
    R = gu.projection_weights(shapes)
    loss = sum((res[k] * torch.tensor(R[k])).sum() for k in sorted(R))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(data["loss"]), rtol=1e-4)
    params = dict(p)
    if emb_t is not None:
        params["t.weight"] = emb_t
    if any(k.startswith("grad_") for k in data):
        for n, t in params.items():
            g = t.grad.numpy() if t.grad is not None else np.zeros(tuple(t.shape), np.float32)
            gu.assert_close("grad " + n, g, data["grad_" + n], rtol=1e-4, atol_frac=1e-5)
    else:
        Q = gu.param_projections([(n, tuple(t.shape)) for n, t in params.items()])
        for n, t in params.items():
            proj = float((t.grad.double() * torch.tensor(Q[n]).double()).sum())
            np.testing.assert_allclose(proj, float(data["gproj_" + n]), rtol=1e-3, atol=1e-6 * float(data["gnorm_" + n]),
                                       err_msg=n)


def test_oracle_sampling_units():
    with np.load(f"{gu.GOLDEN}/unit_sampling.npz") as z:
        d = {k: z[k] for k in z.files}
    s3 = ref_cpu.sample_3sigma(torch.tensor(d["low"]), torch.tensor(d["high"]), 64, torch.tensor(0.0),
                               torch.tensor(0.21), torch.tensor(d["u3"]))
    gu.assert_close("sample_3sigma", s3.numpy(), d["s3"], rtol=1e-6, atol_frac=1e-7)
    sp = ref_cpu.sample_pdf(torch.tensor(d["bins"]), torch.tensor(d["w"]), torch.tensor(d["u_pdf"]))
    gu.assert_close("sample_pdf", sp.numpy(), d["s_pdf"], rtol=1e-6, atol_frac=1e-7)


def test_oracle_composite_unit():
    with np.load(f"{gu.GOLDEN}/unit_composite.npz") as z:
        d = {k: z[k] for k in z.files}
    raw = torch.tensor(d["raw"], requires_grad=True)
    rgb, depth, w, trans = ref_cpu.composite(raw, torch.tensor(d["z"]), torch.tensor(d["noise"]), float(d["noise_std"]))
    for k, v in dict(rgb=rgb, depth=depth, weights=w, transparency=trans).items():
        gu.assert_close(k, v.detach().numpy(), d["out_" + k], rtol=1e-6, atol_frac=1e-7)
    sem = raw[..., 8:].mean(1)
    res = dict(rgb=rgb, depth=depth, weights=w, transparency=trans, albedo=raw[..., :3], sun=raw[..., 4:5],
               sky=raw[..., 5:8], sem_logits=sem)
    R = gu.projection_weights({k: tuple(v.shape) for k, v in res.items()})
    sum((res[k] * torch.tensor(R[k])).sum() for k in sorted(R)).backward()
    gu.assert_close("grad_raw", raw.grad.numpy().reshape(d["grad_raw"].shape), d["grad_raw"], rtol=1e-5, atol_frac=1e-7)
