"""Training parity in PSNR (BASELINE.json metric "PSNR vs ref", north star: within 0.05 dB) —
needs an MI355X.  The HIP path and the pinned CPU restatement of the reference train the same
network from the same init on the same batches and draws, then render the same held-out rays
(bench.psnr_parity; JAX_214 images are not available, so the scene is the synthetic
JAX_269-camera one)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_training_psnr_matches_cpu_reference():
    import bench
    r = bench.psnr_parity(steps=20, batch=128, n_eval=512)
    print(r)
    assert r["loss_first_last"][-1][0] < r["loss_first_last"][0][0]  # it trains
    assert abs(r["delta_db"]) <= 0.05, r
