set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
timeout -k 10 400 python -u -m pytest tests/test_gpu_reuse.py tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r1/t1.log 2>&1 || { echo "T1 FAILED"; grep -E "FAILED|Error|error" gpurun_out/r1/t1.log | head -20; tail -30 gpurun_out/r1/t1.log; exit 1; }
grep -E "difference|bf16 outputs|passed|failed" gpurun_out/r1/t1.log | tail -12
timeout -k 10 500 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_graph.py tests/test_gpu_bf16.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r1/t2.log 2>&1 || { echo "T2 FAILED"; grep -E "FAILED|Error" gpurun_out/r1/t2.log | head -20; tail -30 gpurun_out/r1/t2.log; exit 1; }
tail -1 gpurun_out/r1/t2.log
bash tools/ab_args.sh "" "--no-reuse-pass1"
EXTRA="--global-batch 512" bash tools/ab_args.sh "" "--no-reuse-pass1"
