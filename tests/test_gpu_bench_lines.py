"""The bench's own multi-rank and secondary paths on one MI355X (bench.py, imported and run as
a child process): the row-sharded whole-image C5 render gathered from two ranks equals the
single-process image bit for bit; the default line carries the C5 secondary with its roofline
and MLP MFMA utilisation; and the N>1 gradient path rehearsed with a one-rank RCCL group (the
bucket all-reduces captured into the step graph) reports its exposed collective."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS = 4.0      # the C5 camera at img_downscale 4: 203 x 198 rays (C5 itself renders it at 0.2)
CHUNK = 8192


def _image(rank, world):
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda", 0)
    c = bench.CONFIGS["c5"]
    rays, sems, model, args, h, w, r0 = bench.c5_shard(c, rank, world, dev, img_downscale=DS)
    info = bench.full_image(rays, sems, model, args, CHUNK, rank, world, dev, h, w, c, r0, return_image=True)
    return info


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from spnerf_amd import dp
    torch.cuda.set_device(0)
    dp.init_from_env("gloo")
    info = _image(rank, world)
    if rank == 0:
        np.save(os.path.join(outdir, "image.npy"), info["image"].cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_c5_row_sharded_image_equals_single_process(tmp_path):
    """bench.full_image: two ranks (gloo, sharing cuda:0) each render their image rows in
    8192-ray chunks and all_gather to rank 0; the gathered rgb + depth image equals one process
    rendering every row, bit for bit (draws keyed by the global ray id, labels a function of it)."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "image.npy")
    ref = _image(0, 1)["image"].cpu().numpy()
    assert got.shape == ref.shape and ref.shape[2] == 4 and ref.shape[0] > 100
    assert np.isfinite(ref).all()
    assert np.array_equal(got, ref), float(np.abs(got - ref).max())


def _bench(tag, *args, timeout=110, budget=True):
    """bench.py as a child process; its stdout / stderr kept under gpurun_out/ for diagnosis.  The
    printed line must fit the driver's parse budget (bench.LINE_BUDGET)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", SPNERF_STEP_DEADLINE="90")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"bench_{tag}.out"), "w") as f:
        f.write(p.stdout)
    with open(os.path.join(out, f"bench_{tag}.err"), "w") as f:
        f.write(p.stderr)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    if budget:
        sys.path.insert(0, ROOT)
        import bench
        assert len(line) <= bench.LINE_BUDGET, len(line)
    return json.loads(line)


def test_bench_default_line_carries_c5_secondary():
    """The default line's path at a small batch with EVERY leg on (C4, the C2 and C5 secondaries,
    a short CPU baseline, the psnr_parity legs and a one-seed PSNR study with its side file): the
    line fits the parse budget and carries roofline, cpu_baseline, the study's summary and the C5
    secondary with its roofline and MLP MFMA utilisation."""
    detail = os.path.join(ROOT, "gpurun_out", "psnr_detail_test.json")
    d = _bench("secondary", "--global-batch", "512", "--steps", "3", "--warmup", "2", "--prof-steps", "1",
               "--cpu-seconds", "1", "--cpu-batch", "32", "--psnr-parity-steps", "3", "--psnr-steps", "20",
               "--psnr-seeds", "1", "--psnr-detail", detail, timeout=300)
    assert d["finite"] and d["n_gpus"] == 1 and d["allreduce"] is None
    assert d["roofline"]["frac"] > 0 and d["cpu_baseline"]["value"] > 0
    assert set(d["psnr_parity"]) == {"fp32", "bf16"}
    ps = d["psnr_seeds"]
    assert ps["n_seeds"] == 1 and "worst_grad_checkpoint" in ps and "gradient_gates" in ps
    with open(detail) as f:
        assert "loss_trace_every_10" in json.load(f)["per_seed"][0]
    c5 = d["secondary"]["c5"]
    assert c5["value"] > 0 and c5["roofline"]["frac"] > 0 and c5["mlp_mfma_utilisation"]["frac"] > 0.2
    assert d["secondary"]["c2"]["value"] > 0


def test_bench_line_rehearsed_collective():
    """bench.py at N=1 with --rehearse-collective: a one-rank RCCL group, the bucket all-reduces
    captured into the step graph and replayed; then the profiled eager steps (eager collectives),
    a SECOND capture without the buckets and paired replays of both graphs — round 5's faulting
    sequence, safe since the captured packed-weight buffers live with their graphs.  The exposed
    collective comes from the paired replays (a number, not null), the eager-step figure beside it."""
    d = _bench("rehearse", "--rehearse-collective", "--no-secondary", "--global-batch", "512", "--steps", "3",
               "--warmup", "2", "--prof-steps", "2", "--no-cpu-baseline")
    assert d["finite"] and d["n_gpus"] == 1
    assert "inside the HIP graph" in d["allreduce"], d["allreduce"]
    assert isinstance(d["allreduce_ms_per_step"], float) and d["allreduce_ms_per_step"] >= 0.0
    pr = d["allreduce_exposed_paired_replays"]
    assert pr is not None and pr["replay_ms_with_buckets"] > 0 and pr["replay_ms_without"] > 0
    assert isinstance(d["allreduce_ms_eager_steps"], float)
