"""The bench line stays parsable: every record rank 0 prints is held to bench.LINE_BUDGET bytes
(CPU only).  Round 5's default line grew to 68 KB — per-seed loss traces of the PSNR study — and
the driver did not parse it; these tests rebuild lines of run_train's shape, including that very
record (profiles/r05/bench_default.json), and check the budget and the fields the driver reads."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

R05 = os.path.join(ROOT, "profiles", "r05", "bench_default.json")
HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _check(line: dict, src: dict):
    text = json.dumps(line)
    assert len(text) <= bench.LINE_BUDGET, len(text)
    back = json.loads(text)
    for k in HEADLINE:
        assert k in back, k
    assert back["steps"] == src["steps"] and back["warmup"] == src["warmup"] and back["n_gpus"] == src["n_gpus"]
    assert abs(back["value"] - src["value"]) <= 1e-4 * src["value"]
    assert abs(back["ms_per_step"] - src["ms_per_step"]) <= 1e-4 * src["ms_per_step"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in back["roofline"], k
    assert back["roofline"]["frac"] == pytest.approx(src["roofline"]["frac"], rel=1e-4)
    if "cpu_baseline" in src:
        for k in ("value", "unit", "cores", "kind", "sample"):
            assert k in back["cpu_baseline"], k
    for name, sec in src.get("secondary", {}).items():
        got = back["secondary"][name]
        assert got["value"] == pytest.approx(sec["value"], rel=1e-4)
        assert got["roofline"]["frac"] == pytest.approx(sec["roofline"]["frac"], rel=1e-4)
        assert got["mlp_mfma_utilisation"]["frac"] == pytest.approx(sec["mlp_mfma_utilisation"]["frac"], rel=1e-4)
    return back


def test_round5_line_fits_the_budget():
    """The 68 KB round-5 record itself, finalized: within budget, every headline field, the
    roofline, cpu_baseline and both secondaries intact, the PSNR study reduced to its summary."""
    with open(R05) as f:
        src = json.load(f)
    assert len(json.dumps(src)) > 60000          # the unparsed line
    back = _check(bench.finalize_line(src), src)
    ps = back["psnr_seeds"]
    assert ps["n_seeds"] == 6
    assert "loss_trace_every_10" not in json.dumps(ps) and "grad_floors" not in json.dumps(ps)
    # the worst checkpoint is the one the r05 record names (seed 6, step 250, 0.102)
    w = ps["worst_grad_checkpoint"]
    assert (w["seed"], w["step"]) == (6, 250) and w["grad_rel_err"] == pytest.approx(0.10194, rel=1e-3)
    assert ps["seeds_ending_in_a_loss_spike"] == [4, 7, 8]


def test_synthetic_worst_case_line_fits_the_budget():
    """A line of run_train's shape with every optional leg at its largest (24 kernel classes, a
    12-seed study with 1000-step traces, long strings): trimmed in the documented order, never
    below the headline, roofline, cpu_baseline and secondaries."""
    with open(R05) as f:
        src = json.load(f)
    kern = {f"kernel_class_{i:02d}": {"launches": 33 + i, "ms_per_step": 0.123456789 * i, "avg_us": 17.3456789,
                                      "tflops": 123.456789, "gbs": 3881.831319416358} for i in range(24)}
    src["kernels"] = kern
    seeds = src["psnr_seeds"]
    seeds["per_seed"] = [dict(seeds["per_seed"][0], seed=3 + i) for i in range(12)]
    seeds["n_seeds"] = 12
    src["parity_note"] = src["parity_note"] * 3
    line = bench.finalize_line(src)
    _check(line, src)
    assert "trimmed" in line


def test_compact_rounds_floats_only():
    v = {"a": 1.234567890123, "b": [3, 2.000001, float("inf")], "c": "x", "d": True, "e": 0.0, "f": 12345678}
    got = bench.compact(v)
    assert got == {"a": 1.2346, "b": [3, 2.0, float("inf")], "c": "x", "d": True, "e": 0.0, "f": 12345678}
