set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_graph.py tests/test_gpu_bf16.py tests/test_gpu_variants.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2/t1.log 2>&1 || { echo "T1 FAILED"; grep -E "FAILED|Error|error" gpurun_out/r2/t1.log | head -20; tail -30 gpurun_out/r2/t1.log; exit 1; }
tail -1 gpurun_out/r2/t1.log
bash tools/ab_args.sh "" 
EXTRA="--global-batch 512" bash tools/ab_args.sh ""
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof -o t -- python3 bench.py --config c4 --global-batch 512 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-secondary > gpurun_out/r2/prof.log 2>&1 || exit 1
