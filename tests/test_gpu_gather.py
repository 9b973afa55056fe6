"""spnerf_gather_rows (dp.BatchGather): the training step's per-ray fields gathered in one launch
against torch indexing — bit-exact copies for fp32 / int64 fields of 1, 2, 3 and 11 columns,
repeated and unsorted indices, a one-row batch; and the error for rows that are not a multiple of
4 bytes.  Needs an MI355X."""
import pytest
import torch

import spnerf_amd  # noqa: F401  (the package import path)
from spnerf_amd import dp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _fields(n, g):
    return {
        "rays": torch.randn(n, 11, generator=g).to(DEV),
        "rgbs": torch.rand(n, 3, generator=g).to(DEV),
        "depths": torch.randn(n, 2, generator=g).to(DEV),
        "valid_depth": (torch.rand(n, generator=g) < 0.7).long().to(DEV),
        "depth_std": torch.rand(n, generator=g).to(DEV),
        "sems": torch.randint(-100, 3, (n, 1), generator=g).to(DEV),
    }


@pytest.mark.parametrize("n_src,B", [(10_000, 512), (777, 4096), (5, 1)])
def test_gather_rows_matches_torch_indexing(n_src, B):
    g = torch.Generator(device="cpu").manual_seed(n_src + B)
    f = _fields(n_src, g)
    gather = dp.BatchGather(f, B)
    for step in range(2):   # the static outputs are overwritten by the next batch
        idx = torch.randint(0, n_src, (B,), generator=g).to(DEV)
        out = gather(idx)
        torch.cuda.synchronize()
        for k, t in f.items():
            assert out[k].dtype == t.dtype and out[k].shape == (B,) + tuple(t.shape[1:]), k
            assert torch.equal(out[k], t[idx]), (k, step)


def test_gather_rows_rejects_unaligned_rows():
    with pytest.raises(ValueError):
        dp.BatchGather({"flags": torch.zeros(16, 2, dtype=torch.uint8, device=DEV)}, 4)


def test_gather_rows_poisons_out_of_range_indices():
    """An index outside the source rows (-1, n) poisons its destination row with all-one bits
    (NaN in float fields, -1 in integer ones) — a sampler bug surfaces as a non-finite loss —
    while the in-range rows are exact copies."""
    g = torch.Generator(device="cpu").manual_seed(3)
    f = _fields(100, g)
    gather = dp.BatchGather(f, 6)
    gather(torch.arange(6, device=DEV))          # rows a stale batch would leave behind
    idx = torch.tensor([5, -1, 7, 100, 0, 99], device=DEV)
    out = gather(idx)
    torch.cuda.synchronize()
    bad = torch.tensor([1, 3], device=DEV)
    good = torch.tensor([0, 2, 4, 5], device=DEV)
    for k, t in f.items():
        assert torch.equal(out[k][good], t[idx[good]]), k
        if t.dtype.is_floating_point:
            assert torch.isnan(out[k][bad]).all(), k
        else:
            assert (out[k][bad] == -1).all(), k


def test_rng_begin_advances_and_snapshots():
    """spnerf_rng_begin (PhiloxRandom.begin_render's one launch): the device step advances by one
    per render, the snapshot holds {seed, step} and keeps it while a later render advances the
    state; the host mirror follows; inside a captured graph every replay advances the step."""
    from spnerf_amd import PhiloxRandom
    r = PhiloxRandom(seed=11)
    r.begin_render(DEV)
    s0 = r._snap
    assert r._state.tolist() == [11, 0] and s0.tolist() == [11, 0]
    r.begin_render(DEV)
    assert r._state.tolist() == [11, 1] and r._snap.tolist() == [11, 1] and s0.tolist() == [11, 0]
    assert r.sync_host_step() == 1
    r.reset_step(41)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        r.begin_render(DEV)       # warm-up (eager): step 42
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(g):
        r.begin_render(DEV)       # captured: each replay advances the device step
        snap = r._snap
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert r._state.tolist() == [11, 45] and snap.tolist() == [11, 45]
