# round 3 (session 2): 256x256 TN tiles for 1-3 tile shapes — parity tests, then A/B pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_bf16.py tests/test_gpu_dp.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread -k "few_tiles or tilings or bias_split or bf16 or dp or graph" > gpurun_out/r3j_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3j_tests.log | head -20; tail -5 gpurun_out/r3j_tests.log; exit 1; }
tail -1 gpurun_out/r3j_tests.log
bash tools/gpu_ab_opt.sh "tn_bf16_few_tiles=0" "tn_bf16_few_tiles=1" "tn_bf16_few_tiles=0" "tn_bf16_few_tiles=1"
GB=512 bash tools/ab512.sh "tn_bf16_few_tiles=0" "tn_bf16_few_tiles=1" "tn_bf16_few_tiles=0" "tn_bf16_few_tiles=1"
