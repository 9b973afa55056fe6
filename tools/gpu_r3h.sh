set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flatgrad.py tests/test_gpu_dp.py tests/test_gpu_graph.py > gpurun_out/r3h_test.log 2>&1
bash tools/ab512.sh "" "lib=libspnerf_amd_ds.so" "" "lib=libspnerf_amd_ds.so" > gpurun_out/r3h_ab.log 2>&1
GB=4096 bash tools/ab512.sh "" "lib=libspnerf_amd_ds.so" >> gpurun_out/r3h_ab.log 2>&1
