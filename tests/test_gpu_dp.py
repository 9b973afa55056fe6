"""Config 4 path (BASELINE.json configs[3]: ray-batch data parallelism, one gradient all-reduce
per step) on the HIP kernels — needs an MI355X.

Two ranks share cuda:0 over gloo (RCCL refuses two ranks on one device; the 8-GPU RCCL run is
the driver's).  Each rank renders ITS slice of a shared-seed global batch with the C3 flags
(guided 64+64, solar pass, depth + semantic heads, W=512) through the HIP render path, with the
global batch's first ray as the guided clamp (``clamp_near_far``) and the ignore-index CE
rescaled by ``dp.shard_ce``; then ``dp.allreduce_grads``.  Asserted: both ranks hold the same
gradient, and it equals the single-process gradient of the concatenated batch (reductions over
points run in a different order, hence a tolerance).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

GLOBAL_B, S = 256, 64


class SliceRandom:
    """The render path's random source over per-ray tables of the GLOBAL batch: call k hands
    back rows ``rows`` of table k (stratified u, predicted-window u, GT-window u)."""

    def __init__(self, tables, rows):
        self.tables, self.rows, self.k = tables, rows, 0

    def _take(self, shape, device):
        t = self.tables[self.k][self.rows]
        self.k += 1
        assert tuple(t.shape) == tuple(shape), (t.shape, shape)
        return t.to(device)

    def rand(self, shape, device):
        return self._take(shape, device)

    def noise(self, shape, device, noise_std):
        assert noise_std == 0
        return None

    def gt_uniform(self, valid_mask, n, device):
        return self._take((valid_mask.shape[0], n), device)


def step_grads(rank, world, precision):
    """One C3-flags training step of this rank's slice; returns the (all-reduced) flat gradient."""
    import types
    import spnerf_amd
    from spnerf_amd import dp
    from spnerf_amd.losses import DepthLoss, SemanticLoss, SNerfLoss
    from spnerf_amd.scene import synthetic_scene
    dev = torch.device("cuda", 0)
    scene = synthetic_scene(4.0, seed=0, device=dev)
    sampler = dp.SharedSeedSampler(scene.rays.shape[0], GLOBAL_B, rank, world, seed=5, device=dev)
    gidx, idx = sampler.next()
    b = GLOBAL_B // world
    rows = torch.arange(rank * b, (rank + 1) * b)
    g = torch.Generator().manual_seed(11)
    tables = [torch.rand(GLOBAL_B, S, generator=g) for _ in range(3)]
    torch.manual_seed(0)
    model = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True, precision=precision).to(dev)
    model.use_flat_grads(world > 1)   # the ranks all-reduce the flat buffer in place; one process: autograd
    args = types.SimpleNamespace(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    R = scene
    sem = R.sems[idx]
    with spnerf_amd.random_source(SliceRandom(tables, rows)):
        res = spnerf_amd.render_rays({"coarse": model}, args, R.rays[idx], None, semantics=sem, mode="train",
                                     valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                     target_std=R.depth_std[idx], clamp_near_far=R.rays[gidx[0], 6:8])
    loss = SNerfLoss(lambda_sc=0.1)(res, R.rgbs[idx])[0]
    loss = loss + DepthLoss(1.0, usealldepth=False)(res, R.depths[idx, 0], R.depths[idx, 1], R.valid_depth[idx], R.depth_std[idx])[0]
    sl = SemanticLoss(1.0)(res, sem)[0]
    loss = loss + (dp.shard_ce(sl, sem, R.sems[gidx], world) if world > 1 else sl)
    loss.backward()
    params = list(model.parameters())
    dp.allreduce_grads(params, world)
    return {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()}, gidx.cpu().numpy()


def _worker(rank, world, port, precision, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from spnerf_amd import dp
    torch.cuda.set_device(0)
    dp.init_from_env("gloo")
    grads, gidx = step_grads(rank, world, precision)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), gidx=gidx, **grads)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 5e-3)])
def test_two_ranks_on_hip_equal_single_process(tmp_path, precision, tol):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), precision, str(tmp_path)), nprocs=world, join=True)
    r0 = dict(np.load(tmp_path / "rank0.npz"))
    r1 = dict(np.load(tmp_path / "rank1.npz"))
    assert np.array_equal(r0.pop("gidx"), r1.pop("gidx"))       # same global batch, no collective
    for n in r0:
        assert np.array_equal(r0[n], r1[n]), n                    # identical after the all-reduce
    single, _ = step_grads(0, 1, precision)
    sq_e = sq_r = 0.0
    worst = {}
    for n, ref in single.items():
        e = np.linalg.norm(r0[n].astype(np.float64) - ref) / max(np.linalg.norm(ref), 1e-30)
        sq_e += float(np.sum((r0[n].astype(np.float64) - ref) ** 2))
        sq_r += float(np.sum(ref.astype(np.float64) ** 2))
        if ref.size >= 64 and np.any(ref):
            worst[n] = e
    total = (sq_e / sq_r) ** 0.5
    print(precision, f"flat {total:.2e}", sorted(worst.items(), key=lambda kv: -kv[1])[:4])
    assert total < tol, total
    assert max(worst.values()) < 10 * tol, worst


def render_slice(rank, world, precision="bf16", noise_std=0.0):
    """C3-flags render of this rank's slice of the shared-seed global batch with the production
    random source, spnerf_amd.PhiloxRandom (draws generated inside the kernels, keyed by seed,
    step and GLOBAL ray id: ray_offset = rank · rays per rank); per-ray outputs on the host."""
    import types
    import spnerf_amd
    from spnerf_amd import dp
    from spnerf_amd.scene import synthetic_scene
    dev = torch.device("cuda", 0)
    scene = synthetic_scene(4.0, seed=0, device=dev)
    sampler = dp.SharedSeedSampler(scene.rays.shape[0], GLOBAL_B, rank, world, seed=5, device=dev)
    gidx, idx = sampler.next()
    b = GLOBAL_B // world
    torch.manual_seed(0)
    model = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True, precision=precision).to(dev)
    args = types.SimpleNamespace(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=noise_std)
    R = scene
    outs = []
    with spnerf_amd.random_source(spnerf_amd.PhiloxRandom(seed=11, ray_offset=rank * b)), torch.no_grad():
        for _ in range(2):   # two renders = two steps: the draws must move on
            res = spnerf_amd.render_rays({"coarse": model}, args, R.rays[idx], None, semantics=R.sems[idx], mode="train",
                                         valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                         target_std=R.depth_std[idx], clamp_near_far=R.rays[gidx[0], 6:8])
            outs.append({k: v.detach().cpu().numpy() for k, v in res.items()})
    return outs


def _render_worker(rank, world, port, outdir, noise_std):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from spnerf_amd import dp
    torch.cuda.set_device(0)
    dp.init_from_env("gloo")
    outs = render_slice(rank, world, noise_std=noise_std)
    np.savez(os.path.join(outdir, f"render{rank}.npz"), **{f"{i}|{k}": v for i, o in enumerate(outs) for k, v in o.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("noise_std", [0.0, 0.5])
def test_two_ranks_philox_renders_equal_single_process_bitwise(tmp_path, noise_std):
    """On-device Philox draws keyed by (seed, step, global ray id, slot): two gloo ranks that each
    render half of the global batch produce, ray for ray, exactly the single-process render of the
    whole batch — stratified jitter, guided windows (predicted and GT), σ noise — over two steps,
    with no replayed draw tables; and the second step's draws differ from the first's."""
    world = 2
    mp.spawn(_render_worker, args=(world, _free_port(), str(tmp_path), noise_std), nprocs=world, join=True)
    parts = [dict(np.load(tmp_path / f"render{r}.npz")) for r in range(world)]
    single = render_slice(0, 1, noise_std=noise_std)
    for step, ref in enumerate(single):
        for k, v in ref.items():
            got = np.concatenate([p[f"{step}|{k}"] for p in parts])
            assert got.shape == v.shape, k
            assert np.array_equal(got, v), (step, k, float(np.abs(got - v).max()))
    assert not np.array_equal(single[0]["z_vals_coarse"], single[1]["z_vals_coarse"])


def bucket_runs(rank, world):
    """One C3-flags training step of this rank's slice, three ways, same draws (the Philox
    step is reset before each): eager + the flat all-reduce; eager + dp.GradBuckets (each
    bucket's all-reduce issued behind its backward mark, overlapping the rest of the backward);
    a HIP-graph replay of the step + GradBuckets behind the replay (gloo cannot be captured; with
    RCCL bench.py captures the overlapped buckets into the graph, tools/rccl_capture_probe.py).
    Returns the three reduced flat gradients."""
    import types
    import spnerf_amd
    from spnerf_amd import dp
    from spnerf_amd.losses import FusedRenderLoss
    from spnerf_amd.scene import synthetic_scene
    dev = torch.device("cuda", 0)
    R = synthetic_scene(4.0, seed=0, device=dev)
    sampler = dp.SharedSeedSampler(R.rays.shape[0], GLOBAL_B, rank, world, seed=5, device=dev)
    gidx, idx = sampler.next()
    b = GLOBAL_B // world
    torch.manual_seed(0)
    model = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=512, mapping=True, sem=True,
                              precision="bf16").to(dev).use_flat_grads()
    params = list(model.parameters())
    args = types.SimpleNamespace(n_samples=S, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                 sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)
    floss = FusedRenderLoss(0.1, 1.0, 1.0)
    src = spnerf_amd.PhiloxRandom(seed=11, ray_offset=rank * b)
    buckets = dp.GradBuckets(model, world)

    def fwd_bwd():   # graph-capturable: no host sync (the clamp ray by index_select)
        res = spnerf_amd.render_rays({"coarse": model}, args, R.rays[idx], None, semantics=R.sems[idx], mode="train",
                                     valid_depth=R.valid_depth[idx], target_depths=R.depths[idx],
                                     target_std=R.depth_std[idx],
                                     clamp_near_far=R.rays.index_select(0, gidx[:1])[0, 6:8])
        loss, _ = floss(res, R.rgbs[idx], R.depths[idx], R.valid_depth[idx], R.depth_std[idx], R.sems[idx],
                        labels_global=R.sems[gidx], world=world)
        loss.backward()

    def reset():
        for p in params:
            p.grad = None
        src.reset_step(-1)

    out = []
    with spnerf_amd.random_source(src):
        reset()
        fwd_bwd()
        dp.allreduce_grads(params, world)
        out.append(model._flat_grad.cpu().numpy().copy())
        reset()
        buckets.arm(True)
        fwd_bwd()
        flat = model._flat_grad
        buckets.launch(flat)
        buckets.finish(flat)
        out.append(flat.cpu().numpy().copy())
        # graph: capture on a side stream after the eager warm-up above
        reset()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fwd_bwd()
        flat = model._flat_grad
        src.reset_step(-1)
        graph.replay()
        buckets.launch(flat, overlap=False)   # the replay's marks are the graph's own edges
        buckets.finish(flat)
        out.append(flat.cpu().numpy().copy())
        buckets.arm(False)
    return out


def _bucket_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from spnerf_amd import dp
    torch.cuda.set_device(0)
    dp.init_from_env("gloo")
    flat, bucketed, graphed = bucket_runs(rank, world)
    np.savez(os.path.join(outdir, f"bucket{rank}.npz"), flat=flat, bucketed=bucketed, graphed=graphed)
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_overlapping_the_backward_equals_flat(tmp_path):
    """dp.GradBuckets on the HIP path: the bucket all-reduces wait only for their backward marks
    (spnerf_grad_marks) and run while the rest of the backward does, and give exactly the flat
    all-reduce's gradient (any bucket read before its last write would differ: the backward is
    deterministic); after a graph replay they give it too."""
    world = 2
    mp.spawn(_bucket_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [dict(np.load(tmp_path / f"bucket{r}.npz")) for r in range(world)]
    for p in parts:
        assert np.abs(p["flat"]).max() > 0
        assert np.array_equal(p["bucketed"], p["flat"])
        assert np.array_equal(p["graphed"], p["flat"])
    assert np.array_equal(parts[0]["flat"], parts[1]["flat"])
