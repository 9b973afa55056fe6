set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_parity.py tests/test_gpu_c4.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
REPS=2 bash tools/ab_prev.sh
