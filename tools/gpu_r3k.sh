# round 3 (session 3): narrow N = 512, K = 64 weight-gradient kernel — parity tests, then A/B pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_bf16.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread -k "k64 or skip_layer or bf16 or graph" > gpurun_out/r3k_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3k_tests.log | head -20; tail -5 gpurun_out/r3k_tests.log; exit 1; }
tail -1 gpurun_out/r3k_tests.log
bash tools/gpu_ab_opt.sh "tn_bf16_k64=0" "tn_bf16_k64=1" "tn_bf16_k64=0" "tn_bf16_k64=1"
GB=512 bash tools/ab512.sh "tn_bf16_k64=0" "tn_bf16_k64=1" "tn_bf16_k64=0" "tn_bf16_k64=1"
