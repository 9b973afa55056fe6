set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_c5.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6a_t1.log 2>&1 || { echo "T1 FAILED rc=$?"; tail -40 gpurun_out/r6a_t1.log; exit 1; }
tail -3 gpurun_out/r6a_t1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_lines.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r6a_t2.log 2>&1 || { echo "T2 FAILED rc=$?"; tail -40 gpurun_out/r6a_t2.log; exit 1; }
tail -3 gpurun_out/r6a_t2.log
timeout -k 10 400 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/r6a_bench.err; exit 1; }
wc -c gpurun_out/r6a_bench.json; tail -2 gpurun_out/r6a_bench.err
