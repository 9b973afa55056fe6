set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_graph.py tests/test_gpu_psnr.py > gpurun_out/probe_test.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-device --steps 10 --warmup 3 --no-secondary > gpurun_out/r3d_share2.json 2> gpurun_out/r3d_share2.err
