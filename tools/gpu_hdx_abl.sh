set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -k "heads_dx" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/gpu_ab_opt.sh "heads_dx=0" "heads_dx=1" "heads_dx=0" "heads_dx=1"
