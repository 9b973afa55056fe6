"""Data-parallel path on CPU (gloo, world_size 2): shared-seed sampling, one flat gradient
all-reduce, loss decomposition.  The per-rank compute is the oracle (CPU); the DP logic under
test is sp-nerf_amd/dp.py, the same code bench.py runs over RCCL."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_cpu
from oracle.weights import ModelDims, make_weights
from spnerf_amd import dp

DIMS = ModelDims(width=64)
ARGS = types.SimpleNamespace(n_samples=16, n_importance=0, model="sp-nerf", beta=False, guidedsample=False,
                             sc_lambda=0.05, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
N_RAYS, GB = 96, 32


def _scene():
    rng = np.random.default_rng(0)
    rays = np.zeros((N_RAYS, 11), np.float32)
    rays[:, 0:3] = rng.uniform(-0.5, 0.5, (N_RAYS, 3))
    d = rng.normal(size=(N_RAYS, 3)) + np.array([0, 0, -3.0])
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = 0.2
    rays[:, 9] = 1.0
    rgbs = rng.uniform(0, 1, (N_RAYS, 3)).astype(np.float32)
    u = rng.uniform(size=(N_RAYS, ARGS.n_samples)).astype(np.float32)
    return torch.tensor(rays), torch.tensor(rgbs), torch.tensor(u)


def _step_grads(idx, world):
    """oracle render + the reference colour/solar losses on rays idx → flat gradient."""
    rays, rgbs, u = _scene()
    p = ref_cpu.to_params(make_weights(DIMS, 0), requires_grad=True)
    queue = [("rand", u[idx]), ("randn", torch.zeros(len(idx), ARGS.n_samples)),
             ("randn", torch.zeros(len(idx), ARGS.n_samples))]
    draw = lambda kind, shape: queue.pop(0)[1]
    res = ref_cpu.render_rays(p, DIMS, ARGS, rays[idx], draw=draw)
    sun_sc = res["sun_sc_coarse"].squeeze()
    loss = torch.mean((res["rgb_coarse"] - rgbs[idx]) ** 2)
    loss = loss + 0.05 / 3 * torch.mean(torch.sum((res["transparency_sc_coarse"].detach() - sun_sc) ** 2, -1))
    loss.backward()
    return p


def _cfg(d):
    from spnerf_amd import _lib
    c = _lib.ModelCfg()
    c.width, c.layers, c.skip = d.width, d.layers, d.skips[0]
    c.n_freq = d.n_freq if d.mapping else 0
    c.sem_classes = d.num_sem_classes if d.sem else 0
    c.sem_dim = d.sem_dim
    c.beta, c.t_dim = int(d.beta), (d.t_dim if d.beta else 0)
    return c


def _bucket_worker(rank, world, port, out):
    """the bucketed all-reduce (dp.GradBuckets, marks from the library) vs the flat one"""
    from spnerf_amd import _lib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, _, w = dp.init_from_env("gloo")
    sampler = dp.SharedSeedSampler(N_RAYS, GB, r, w, seed=3)
    _, idx = sampler.next()
    params = list(_step_grads(idx, w).values())
    flat = torch.cat([t.grad.reshape(-1) for t in params])
    marks, n = _lib.grad_marks(_cfg(DIMS), len(params))
    b = dp.GradBuckets(None, w, layout=([t.numel() for t in params], marks))
    bucketed = flat.clone()
    b.launch(bucketed)
    b.finish(bucketed)
    dp.allreduce_grads(params, w)
    out[rank] = (bucketed.numpy(), torch.cat([t.grad.reshape(-1) for t in params]).numpy(), len(b.buckets), n)
    dist.destroy_process_group()


def test_bucketed_allreduce_equals_flat_allreduce():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for rank in range(world):
        bucketed, flat, nb, n_marks = out[rank]
        assert np.array_equal(bucketed, flat)    # same sums (a + b per element), same /world
        assert nb > 8 and n_marks == DIMS.layers + 2
    assert np.array_equal(out[0][0], out[1][0])


@pytest.mark.parametrize("sem", [False, True])
def test_grad_marks_cover_every_parameter_in_backward_order(sem):
    """every parameter gets a mark; trunk layers become final top-down after the heads; the
    per-ray parameters (and the semantic columns of layer 0 / the skip layer) at the end"""
    from spnerf_amd import _lib
    from oracle.weights import param_specs
    d = ModelDims(width=64, sem=sem)
    specs = param_specs(d)
    marks, n = _lib.grad_marks(_cfg(d), len(specs))
    m = {name: k for (name, _, _), k in zip(specs, marks)}
    L, end = d.layers, d.layers + 1
    assert n == L + 2 and min(marks) == 0 and max(marks) == end
    for i in range(L):
        assert m[f"fc_net.{2 * i}.bias"] == 1 + (L - 1 - i)
        sem_cols = sem and i in (0, d.skips[0])
        assert m[f"fc_net.{2 * i}.weight"] == (end if sem_cols else 1 + (L - 1 - i))
    assert m["sigma_from_xyz.0.weight"] == m["feats_from_xyz.weight"] == m["sun_v_net.2.weight"] == 0
    assert m["sun_v_net.0.weight"] == m["sky_color.0.weight"] == end
    numels = [int(np.prod(s)) for _, s, _ in specs]
    b = dp.bucket_ranges(numels, marks)
    covered = sorted((lo, hi) for _, lo, hi in b)
    assert covered[0][0] == 0 and covered[-1][1] == sum(numels)
    assert all(a[1] == c[0] for a, c in zip(covered, covered[1:]))
    assert [k for k, _, _ in b] == sorted(k for k, _, _ in b)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, _, w = dp.init_from_env("gloo")
    sampler = dp.SharedSeedSampler(N_RAYS, GB, r, w, seed=3)
    gidx, idx = sampler.next()
    p = _step_grads(idx, w)
    params = list(p.values())
    dp.allreduce_grads(params, w)
    flat = torch.cat([t.grad.reshape(-1) for t in params])
    gathered = [torch.empty_like(gidx) for _ in range(w)]
    dist.all_gather(gathered, gidx)
    out[rank] = (flat.numpy(), gidx.numpy(), torch.stack(gathered).numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_dp_two_ranks_gradient_equals_single_process():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, gidx0, all0 = out[0]
    g1, gidx1, _ = out[1]
    # every rank drew the same global batch (no collective needed to agree on it)
    assert np.array_equal(gidx0, gidx1)
    assert np.array_equal(all0[0], all0[1])
    # after the all-reduce both ranks hold the same gradient ...
    np.testing.assert_allclose(g0, g1, rtol=0, atol=0)
    # ... equal to the single-process gradient of the concatenated batch (mean losses decompose)
    p = _step_grads(torch.tensor(gidx0), 1)
    ref = torch.cat([t.grad.reshape(-1) for t in p.values()]).numpy()
    np.testing.assert_allclose(g0, ref, rtol=2e-4, atol=1e-7 * np.abs(ref).max())


def test_shared_seed_sampler_partitions_each_global_batch():
    s = [dp.SharedSeedSampler(100, 20, r, 4, seed=1) for r in range(4)]
    for _ in range(12):   # crosses epoch boundaries
        parts = [x.next() for x in s]
        g = parts[0][0]
        assert all(torch.equal(p[0], g) for p in parts)
        assert torch.equal(torch.cat([p[1] for p in parts]), g)
        assert len(set(g.tolist())) == 20


def test_cross_entropy_rescale_recovers_global_mean():
    torch.manual_seed(0)
    logits = torch.randn(40, 3)
    labels = torch.randint(0, 3, (40,))
    labels[::5] = -100
    ce = torch.nn.CrossEntropyLoss(ignore_index=-100)
    glob = ce(logits, labels)
    parts = []
    for r in range(4):
        sl = slice(10 * r, 10 * r + 10)
        parts.append(dp.ce_scale(labels[sl], labels, 4) * ce(logits[sl], labels[sl]))
    np.testing.assert_allclose(float(sum(parts) / 4), float(glob), rtol=1e-6)


def test_shard_ce_handles_a_shard_without_labels():
    """A rank whose slice is all ignore_index (local CE = NaN) contributes 0, and the shards
    still recover the global mean; the scale stays on the device (no host sync)."""
    torch.manual_seed(1)
    logits = torch.randn(40, 3)
    labels = torch.randint(0, 3, (40,))
    labels[:10] = -100                      # shard 0 has no valid label
    ce = torch.nn.CrossEntropyLoss(ignore_index=-100)
    glob = ce(logits, labels)
    parts = [dp.shard_ce(ce(logits[10 * r:10 * r + 10], labels[10 * r:10 * r + 10]), labels[10 * r:10 * r + 10],
                         labels, 4) for r in range(4)]
    assert torch.is_tensor(dp.ce_scale(labels[:10], labels, 4))
    assert torch.isfinite(parts[0]) and float(parts[0]) == 0.0
    np.testing.assert_allclose(float(sum(parts) / 4), float(glob), rtol=1e-6)


_STALL_SCRIPT = r"""
import os, sys, time
sys.path.insert(0, os.environ["SPN_ROOT"])
import torch, torch.distributed as dist
from spnerf_amd import dp
r, _, w = dp.init_from_env("gloo")
wd = dp.StepWatchdog(rank=r, mode="test", deadline=3.0, poll=0.2,
                     probe=lambda: {"buckets_done": [0, 1]})
x = torch.ones(4)
for step in range(6):
    wd.beat(step, "timed")
    if r == 1 and step == 2:
        time.sleep(60)          # the injected stall: rank 0 waits in the collective
    dist.all_reduce(x)
wd.close()
print("finished", flush=True)
"""


def test_step_watchdog_ends_a_stalled_rank_with_a_diagnosis():
    """A rank that stalls mid-loop (and the rank blocked in the collective behind it) exits
    non-zero within the step deadline, printing one JSON diagnosis (rank, step, phase) instead of
    hanging until the process group's timeout (dp.StepWatchdog, used by bench.py's loops)."""
    import json
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(2):
        env = dict(os.environ, SPN_ROOT=root, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-c", _STALL_SCRIPT], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=45)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("the watchdog did not end the stalled job")
        outs.append((p.returncode, o, e))
    assert time.monotonic() - t0 < 40
    for r, (code, o, e) in enumerate(outs):
        assert code == 3, (r, code, o, e[-2000:])
        line = [ln for ln in o.splitlines() if ln.startswith("{")][-1]
        d = json.loads(line)
        assert d["watchdog"] == "step deadline exceeded" and d["rank"] == r and d["step"] == 2, d
        assert d["phase"] == "timed" and d["buckets_done"] == [0, 1] and d["seconds_since_beat"] >= 3.0
        assert "finished" not in o
