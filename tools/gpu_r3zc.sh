# round 3 (session 3): the per-ray sky-gradient sum in parallel — parity tests, A/B against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3zc_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3zc_tests.log | head -20; tail -5 gpurun_out/r3zc_tests.log; exit 1; }
tail -1 gpurun_out/r3zc_tests.log
GB=512 bash tools/ab512.sh "lib=libspnerf_amd_prev.so" "trunk_nt=1" "lib=libspnerf_amd_prev.so" "trunk_nt=1"
CFG=c4 bash tools/pmc_clock.sh > gpurun_out/pmc_c4_final.txt 2>&1 || { tail -20 gpurun_out/pmc_c4_final.txt; exit 1; }
head -40 gpurun_out/pmc_c4_final.txt
