"""sha256 of the flat gradient (and loss) of one eager C4 training step at a fixed seed: run it
under two library builds (SPNERF_AMD_LIB=...) to show a kernel change is bit-identical.

    python tools/grad_hash.py [--global-batch 512] [--config c3]
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    cfg = "c4"
    if "--config" in argv:
        k = argv.index("--config")
        cfg = argv[k + 1]
        argv = argv[:k] + argv[k + 2:]
    a = bench.parse_args(argv + ["--no-cpu-baseline", "--no-secondary"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ts = bench.TrainStep(a, cfg, 0, 1, dev)
    ts.load_batch()
    ts.opt.zero_grad(set_to_none=True)
    loss = ts.fwd_bwd()
    torch.cuda.synchronize()
    g = ts.model._flat_grad.detach().cpu().numpy().tobytes()
    print(f"{os.environ.get('SPNERF_AMD_LIB', 'libspnerf_amd.so')} {cfg} B={ts.B} loss={float(loss):.9g} "
          f"grad_sha={hashlib.sha256(g).hexdigest()[:16]} rgb_sha="
          f"{hashlib.sha256(ts.res['rgb_coarse'].detach().cpu().numpy().tobytes()).hexdigest()[:16]}")
    ts.close()


if __name__ == "__main__":
    main()
