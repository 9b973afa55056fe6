set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/h1
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -k "heads_dx" -x -v --timeout 200 --timeout-method thread > gpurun_out/h1/t.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/h1/t.log | head -20; tail -30 gpurun_out/h1/t.log; exit 1; }
tail -1 gpurun_out/h1/t.log
bash tools/ab_opt_pairs.sh "heads_dx=0" "heads_dx=1"
EXTRA="--global-batch 512" bash tools/ab_opt_pairs.sh "heads_dx=0" "heads_dx=1"
