set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_trunk.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
CONFIG=c5 bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so" "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so"
