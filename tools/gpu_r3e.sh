# trunk copy-outs through buffer descriptors: bit-exactness tests, then A/B against the guarded-store build
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trunk.py tests/test_gpu_variants.py tests/test_gpu_bf16.py > gpurun_out/r3e_test.log 2>&1
bash tools/ab512.sh "" "lib=libspnerf_amd_gs.so" "" "lib=libspnerf_amd_gs.so" > gpurun_out/r3e_ab.log 2>&1
GB=4096 bash tools/ab512.sh "" "lib=libspnerf_amd_gs.so" "" "lib=libspnerf_amd_gs.so" >> gpurun_out/r3e_ab.log 2>&1
