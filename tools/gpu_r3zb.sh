# round 3 (session 3): σ rows from the training trunk (trunk_sigma) — bitwise tests, A/B pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py tests/test_gpu_bf16.py tests/test_gpu_variants.py -x -v --timeout 200 --timeout-method thread -k "trunk or bf16 or backward" > gpurun_out/r3zb_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3zb_tests.log | head -20; tail -5 gpurun_out/r3zb_tests.log; exit 1; }
tail -1 gpurun_out/r3zb_tests.log
bash tools/gpu_ab_opt.sh "trunk_sigma=0" "trunk_sigma=1" "trunk_sigma=0" "trunk_sigma=1"
GB=512 bash tools/ab512.sh "trunk_sigma=0" "trunk_sigma=1" "trunk_sigma=0" "trunk_sigma=1"
