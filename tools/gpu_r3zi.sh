# round 3 (session 3): bias reads hoisted out of the register-D epilogue's point-tile loop (SPN_BIAS_HOIST) — bitwise tests, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3zi_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3zi_tests.log | head -20; tail -5 gpurun_out/r3zi_tests.log; exit 1; }
tail -1 gpurun_out/r3zi_tests.log
for lib in libspnerf_amd_nohoist.so libspnerf_amd.so libspnerf_amd_nohoist.so libspnerf_amd.so; do
echo "== $lib"; SPNERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 --option trunk_var=0 2>&1 | grep save || exit 1
done
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_nohoist.so" "trunk_var=0" "lib=libspnerf_amd_nohoist.so" "trunk_var=0"
