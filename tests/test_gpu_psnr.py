"""Training parity in PSNR (BASELINE.json metric "PSNR vs ref", north star: within 0.05 dB) —
needs an MI355X.  The HIP path and the pinned CPU restatement of the reference train the same
network from the same init on the same batches and draws, then render the same held-out rays
(bench.psnr_parity: the JAX_269 cameras at img_downscale 4 with the real JAX_269 images as
targets; JAX_214 is not available), for the fp32 MLP and for the bf16 MLP of configs 3-5."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_training_psnr_matches_cpu_reference(precision):
    import bench
    r = bench.psnr_parity(steps=20, batch=128, n_eval=512, precision=precision)
    print(r)
    assert r["targets"] == "real JAX_269 RGB"
    assert r["loss_first_last"][-1][0] < r["loss_first_last"][0][0]  # it trains
    assert abs(r["delta_db"]) <= 0.05, r


def test_long_horizon_bf16_psnr_matches_fp32_hip():
    """bench.psnr_long at a test-sized horizon (the default bench line runs 2000 steps of 1024
    rays): fp32, bf16 and an fp32 control (init x (1 + 1e-6 N(0,1))) trained side by side with the
    C3 flags on the real JAX_269 targets, same batches / on-device draws.  Trajectory noise makes
    the trained-PSNR difference of ANY two runs (the control shows it) exceed 0.05 dB at long
    horizons, so the precision claims are held where they are resolvable: the fp32-trained weights
    rendered by the bf16 MLP within 0.05 dB, and the bf16 gradient at the fp32 trajectory's weights
    close at every checkpoint."""
    import bench
    r = bench.psnr_long(steps=300, batch=256, n_eval=2048, checkpoints=6)
    print({k: v for k, v in r.items() if k not in ("loss_curve", "psnr_curve")})
    assert r["targets"] == "real JAX_269 RGB"
    for arm in ("fp32", "bf16", "fp32_control"):
        curve = r["loss_curve"][arm]
        assert curve[-1][1] < curve[0][1]   # every arm trains
    assert abs(r["bf16_inference_at_fp32_trained"]["delta_db"]) <= 0.05, r
    # at init the fixtures' bf16 bound (0.4% measured at 256 rays); along the run the
    # norm-relative error grows where the gradient shrinks and cancels over the batch — the worst
    # tensors are the sun-visibility head's — so the run is held to the bench's
    # gradient gates (bench.GRAD_GATES, the same ones the bench line evaluates over 6 seeds x 8
    # checkpoints): median and max of that error, and the max of its ratio to the fp32 gradient's
    # own change between two batches at the same weights (the minibatch noise)
    import numpy as np
    assert r["grad_rel_err"][0][1] <= 2e-2, r["grad_rel_err"]
    errs = np.array([e for _, e in r["grad_rel_err"]])
    ratios = np.array([e / f["other_batch"] for (_, e), f in zip(r["grad_rel_err"], r["grad_floors"])])
    gates = bench.grad_gates(errs, ratios)
    print("gates", gates, "floors", r["grad_floors"])
    assert all(g["pass"] for g in gates.values()), gates
    # the trained-PSNR difference of two trajectories is reported (with the control beside it,
    # and as paired multi-seed statistics in the bench line: bench.psnr_seeds), not gated: at this
    # horizon it measures trajectory noise, not precision
    print("trained delta", r["delta_db"], "control", r["control_delta_db"])
