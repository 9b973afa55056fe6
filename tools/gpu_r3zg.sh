# round 3 (session 3): weight-gradient options re-measured with tn_bf16_ip 1; the TN tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_graph.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3zg_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3zg_tests.log | head -20; tail -5 gpurun_out/r3zg_tests.log; exit 1; }
tail -1 gpurun_out/r3zg_tests.log
bash tools/gpu_ab_opt.sh "trunk_nt=1" "tn_bf16_bias_split=0" "tn_bf16_few_tiles=0" "tn_bf16_min_points=2048" "trunk_nt=1" "tn_bf16_bias_split=0" "tn_bf16_few_tiles=0" "tn_bf16_min_points=2048"
