set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/m1
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/m1/t.log 2>&1 || { tail -30 gpurun_out/m1/t.log; exit 1; }
tail -1 gpurun_out/m1/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m1/prof -o t -- python3 bench.py --config c4 --global-batch 512 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-secondary > gpurun_out/m1/prof.log 2>&1 || exit 1
