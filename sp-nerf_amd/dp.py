"""Ray-batch data parallelism (one process per GPU, torch.distributed over RCCL/xGMI).

The reference is single-GPU (main.py:322-337).  Rays are independent, so each rank renders
its slice of the global batch with replicated weights and the only collective is ONE
all-reduce of the flat gradient bucket per step (2.70 M fp32 params = 10.8 MB).

Parity under sharding:
* every rank draws the SAME global permutation (shared-seed sampler), so each knows the
  global batch without a collective;
* the guided-sampling clamp uses the chunk's first ray (rendering.py:95,113): ranks pass the
  global batch's ray-0 near/far through ``render_rays(..., clamp_near_far=...)``;
* losses that are means over the batch decompose into per-rank means when every rank has
  B/N rays; cross-entropy with ignore_index does not (it averages over valid labels), so it is
  rescaled by local_valid / global_valid (``ce_scale``).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def pg_timeout_seconds() -> float:
    """Collective timeout of the process group: SPNERF_PG_TIMEOUT seconds (default 300).  A
    collective that does not complete in that time aborts the rank (RCCL's watchdog) instead of
    hanging the job — a step is milliseconds, so minutes mean a deadlock."""
    return float(os.environ.get("SPNERF_PG_TIMEOUT", "300"))


def init_from_env(backend: str = "nccl", device=None):
    """Join the process group torchrun describes in the environment.  Call it AFTER
    ``torch.cuda.set_device``; with RCCL the rank's device is bound eagerly (``device_id``).
    Every group gets a finite ``timeout`` (``pg_timeout_seconds``)."""
    import datetime
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": torch.device(device)} if (backend == "nccl" and device is not None) else {}
        if backend == "nccl":
            # fail fast: a hung collective raises on the host instead of waiting forever
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=pg_timeout_seconds()), **kw)
    return rank, local, world


def step_deadline_seconds() -> float:
    """Host-side deadline of one step of a timed loop: SPNERF_STEP_DEADLINE seconds (default 120;
    0 = off).  A C4 step is tens of milliseconds, so a step still running after minutes is a hang."""
    return float(os.environ.get("SPNERF_STEP_DEADLINE", "120"))


class StepWatchdog:
    """Make a hung step end the process with a diagnosis instead of blocking until the driver's
    limit.  The loop calls ``beat(step, phase)`` before each step and ``mark(event)`` after it
    (an optional CUDA event recorded behind the step's work); a daemon thread checks once a
    second, and when no beat came for ``deadline`` seconds it prints ONE JSON line (rank, step,
    phase, mode, seconds since the beat, the last step whose event had completed, and the
    optional ``probe()`` dict, e.g. which gradient buckets' marks had fired) to stdout and stderr
    and calls ``os._exit(code)`` — a non-zero exit of THIS process (never a re-exec), which
    torchrun turns into the job's failure.  The GIL is released while the main thread blocks in
    a device synchronize or a collective, so the thread runs then."""

    def __init__(self, rank: int = 0, mode: str = "", deadline: float | None = None, code: int = 3, probe=None,
                 poll: float = 1.0):
        import threading
        self.rank, self.mode, self.code, self.probe, self.poll = rank, mode, code, probe, poll
        self.deadline = step_deadline_seconds() if deadline is None else float(deadline)
        self.step, self.phase = -1, "start"
        self.events = []       # (step, event) of the steps marked so far (the last few)
        self._t = None
        self._stop = threading.Event()
        self._last = None
        if self.deadline > 0:
            import time
            self._last = time.monotonic()
            self._t = threading.Thread(target=self._run, name="spnerf-step-watchdog", daemon=True)
            self._t.start()

    def beat(self, step: int, phase: str) -> None:
        import time
        self.step, self.phase = step, phase
        self._last = time.monotonic()

    def mark(self, event) -> None:
        self.events = (self.events + [(self.step, event)])[-4:]

    def _completed(self):
        done = None
        for st, ev in list(self.events):
            try:
                if ev.query():
                    done = st
            except Exception:   # a faulted device: the query itself fails
                return "query failed"
        return done

    def diagnosis(self) -> dict:
        import time
        d = {"watchdog": "step deadline exceeded", "rank": self.rank, "step": self.step, "phase": self.phase,
             "mode": self.mode, "seconds_since_beat": round(time.monotonic() - self._last, 1),
             "deadline_s": self.deadline, "last_completed_step": self._completed()}
        if self.probe is not None:
            try:
                d.update(self.probe())
            except Exception as e:   # the diagnosis must not fail
                d["probe_error"] = f"{type(e).__name__}: {e}"
        return d

    def _run(self):
        import json
        import sys
        import time
        while not self._stop.wait(self.poll):
            if time.monotonic() - self._last > self.deadline:
                line = json.dumps(self.diagnosis())
                print(line, flush=True)
                print(line, file=sys.stderr, flush=True)
                os._exit(self.code)

    def close(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2 * self.poll + 1)


class SharedSeedSampler:
    """Every rank draws the same permutation of the N training rays per epoch (uniform
    shuffle, main.py:108-115) and takes rows [rank·b, (rank+1)·b) of each global batch."""

    def __init__(self, n_rays: int, global_batch: int, rank: int, world: int, seed: int = 0, device="cpu"):
        assert global_batch % world == 0, "global batch must divide over ranks"
        self.n, self.gb, self.rank, self.world = n_rays, global_batch, rank, world
        self.local = global_batch // world
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self.device = device
        self.perm = None
        self.pos = n_rays

    def next_global(self) -> torch.Tensor:
        if self.pos + self.gb > self.n:
            self.perm = torch.randperm(self.n, generator=self.gen).to(self.device)
            self.pos = 0
        idx = self.perm[self.pos:self.pos + self.gb]
        self.pos += self.gb
        return idx

    def next(self):
        """(global indices, this rank's indices)"""
        g = self.next_global()
        return g, g[self.rank * self.local:(self.rank + 1) * self.local]


class BatchGather:
    """The batch's per-ray fields gathered in ONE launch (spnerf_gather_rows) into buffers
    allocated once: ``out[k][i] = fields[k][idx[i]]`` for every key — the trainer's
    ``batch[k]`` from the DataLoader (main.py:108-115, satellite_scene.py:577-592), with the
    dataset resident in HBM.  Bit-exact copies; the static outputs let a captured HIP graph read
    each new batch.  Every field: contiguous on the GPU, rows a multiple of 4 bytes, at most 8."""

    def __init__(self, fields: dict, n: int):
        import ctypes
        from . import _lib
        self._lib = _lib
        self.keys = list(fields)
        assert 0 < len(self.keys) <= 8, "BatchGather: 1..8 fields"
        self.src = [fields[k].contiguous() for k in self.keys]
        _lib.require_device(*self.src)
        self.out = {k: torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
                    for k, t in zip(self.keys, self.src)}
        self.n = n
        nf = len(self.keys)
        row_bytes = [t.element_size() * (t.numel() // max(t.shape[0], 1)) for t in self.src]
        for k, rb in zip(self.keys, row_bytes):
            if rb % 4:
                raise ValueError(f"BatchGather: field {k!r} rows are {rb} bytes (not a multiple of 4)")
        self._src = (ctypes.c_void_p * nf)(*[t.data_ptr() for t in self.src])
        self._dst = (ctypes.c_void_p * nf)(*[self.out[k].data_ptr() for k in self.keys])
        self._rows = (ctypes.c_int64 * nf)(*[t.shape[0] for t in self.src])
        self._rb = (ctypes.c_int32 * nf)(*row_bytes)

    def __call__(self, idx: torch.Tensor) -> dict:
        assert idx.dtype == torch.int64 and idx.is_contiguous() and idx.numel() == self.n, "BatchGather: idx"
        self._lib.require_device(idx)
        self._lib.check(self._lib.lib().spnerf_gather_rows(self._lib.ptr(idx), self.n, len(self.keys), self._src,
                                                          self._rows, self._rb, self._dst, self._lib.stream_of(idx)),
                        "gather_rows")
        return self.out


def allreduce_grads(params, world: int, group=None):
    """One flat all-reduce (SUM then /world) of every gradient.

    Parameters without a gradient stay without one (Adam skips them, as on one GPU).  Which
    parameters have gradients depends only on the model configuration and the render flags, so
    the set is the same on every rank and the flat buffers line up."""
    if world <= 1:
        return
    have = [p for p in params if p.grad is not None]
    if not have:
        return
    grads = [p.grad for p in have]
    flat = _shared_flat(grads)
    if flat is not None:   # the .grads are consecutive views of one buffer (SPNeRF's flat gradient)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        flat.div_(world)
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world)
    for p, g in zip(have, torch._utils._unflatten_dense_tensors(flat, grads)):
        p.grad.copy_(g)


def bucket_ranges(numels, marks):
    """Buckets of a flat gradient laid out in canonical parameter order: maximal runs of
    consecutive parameters that become final at the same backward mark, as (mark, lo, hi)
    element ranges sorted by mark (stable), covering [0, sum(numels)) exactly once."""
    out, off = [], 0
    for n, m in zip(numels, marks):
        if out and out[-1][0] == m and out[-1][2] == off:
            out[-1] = (m, out[-1][1], off + n)
        else:
            out.append((m, off, off + n))
        off += n
    return sorted(out, key=lambda r: r[0])


class GradBuckets:
    """The gradient all-reduce of a flat-gradient SPNeRF split into buckets, each issued as soon
    as the backward has finished writing it, so the collectives overlap the rest of the backward.

    The library's backward records mark events at fixed points (spnerf_grad_marks: after the
    output heads' gradients, after each trunk layer's weight gradient, at the end); parameter p
    is final at mark(p).  ``launch`` makes a communication stream wait for each bucket's mark and
    issues its all_reduce(SUM) there (RCCL runs it on its own stream behind that wait); ``finish``
    makes the current stream wait for every bucket, then divides by the world size.  ``arm``
    must precede the backward.  Under HIP-graph capture the marks are edges of the graph being
    captured, so the overlapped all-reduces must be captured with the backward (RCCL); a graph
    that holds only the backward is followed by ``launch(flat, overlap=False)``."""

    def __init__(self, model, world: int, group=None, layout=None):
        """``layout`` = (numels, marks) instead of the model's (host tests of the bucketing on
        CPU tensors: no mark events, no streams)."""
        from . import _lib
        self._lib = _lib
        self.world, self.group = world, group
        if layout is None:
            params = list(model.parameters())
            numels = [p.numel() for p in params]
            marks, self.n_marks = _lib.grad_marks(model.cfg(), len(params))
        else:
            numels, marks = layout
            self.n_marks = max(marks) + 1
        self.buckets = bucket_ranges(numels, marks)
        self.stream = None
        self.works = []

    def arm(self, on: bool = True) -> None:
        self._lib.grad_marks_arm(on)

    def launch(self, flat: torch.Tensor, overlap: bool = True, force: bool = False) -> None:
        """Issue every bucket's all-reduce.  ``overlap``: behind its backward mark — in the same
        eager step or the same HIP-graph capture as the backward; otherwise (a graph replay's
        backward, whose marks are that graph's internal edges) behind the whole compute stream.
        ``force``: also with one rank (a capture rehearsal of the collective on one GPU)."""
        if self.world <= 1 and not force:
            return
        on_gpu = flat.is_cuda
        if on_gpu and self.stream is None:
            self.stream = torch.cuda.Stream(device=flat.device)
        if on_gpu and not overlap:
            self.stream.wait_stream(torch.cuda.current_stream(flat.device))
        for mark, lo, hi in self.buckets:
            if not on_gpu:
                self.works.append(dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
                continue
            if overlap:
                self._lib.grad_mark_wait(mark, self.stream)
            with torch.cuda.stream(self.stream):
                self.works.append(dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                                  async_op=True))

    def finish(self, flat: torch.Tensor, force: bool = False) -> None:
        if self.world <= 1 and not force:
            return
        for w in self.works:
            w.wait()
        self.works = []
        if self.world > 1:
            flat.div_(self.world)


def _shared_flat(grads):
    """The buffer the gradients are consecutive views of, covering it exactly; else None."""
    base = grads[0]._base
    if base is None or base.dim() != 1 or not base.is_contiguous():
        return None
    ptr, esz = base.data_ptr(), base.element_size()
    off = 0
    for g in grads:
        if g._base is not base or g.data_ptr() != ptr + esz * off or not g.is_contiguous():
            return None
        off += g.numel()
    return base if off == base.numel() else None


def ce_scale(local_labels: torch.Tensor, global_labels: torch.Tensor, world: int) -> torch.Tensor:
    """Factor turning the local ignore_index mean CE into its share of the global mean
    (metrics.py:166 does not decompose over shards; SURVEY §8e pitfall 2).  A 0-d tensor on
    the labels' device — no host sync."""
    lv = (local_labels != -100).sum().to(torch.float32)
    gv = (global_labels != -100).sum().to(torch.float32)
    return torch.where(gv > 0, world * lv / gv.clamp_min(1.0), torch.zeros_like(gv))


def shard_ce(ce_local: torch.Tensor, local_labels: torch.Tensor, global_labels: torch.Tensor, world: int) -> torch.Tensor:
    """``ce_scale · ce_local`` with a shard that holds no valid label contributing 0 (its local
    ignore_index mean is NaN) — the term each rank adds to its loss before the gradient
    all-reduce averages over ranks."""
    scale = ce_scale(local_labels, global_labels, world)
    return torch.where(scale > 0, scale * torch.nan_to_num(ce_local), torch.zeros_like(ce_local))
