# round 3 (session 3): trunk epilogues moving whole 16-B LDS chunks (SPN_LDS128) — bitwise tests, PMC, A/B vs the 8-B build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py tests/test_gpu_variants.py tests/test_gpu_bf16.py -x -v --timeout 200 --timeout-method thread -k "trunk or backward or bf16" > gpurun_out/r3zd_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3zd_tests.log | head -20; tail -5 gpurun_out/r3zd_tests.log; exit 1; }
tail -1 gpurun_out/r3zd_tests.log
for lib in libspnerf_amd_lds64.so libspnerf_amd.so libspnerf_amd_lds64.so libspnerf_amd.so; do
echo "== $lib"; SPNERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 2>&1 | grep save || exit 1
done
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_lds64.so" "trunk_nt=1" "lib=libspnerf_amd_lds64.so" "trunk_nt=1"
GB=512 bash tools/ab512.sh "lib=libspnerf_amd_lds64.so" "trunk_nt=1"
