set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_gputest2.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 gpurun_out/r2_gputest2.log; exit 1; }
tail -3 gpurun_out/r2_gputest2.log
timeout -k 10 400 python bench.py > gpurun_out/r2_bench_default.json 2> gpurun_out/r2_bench_default.err || { echo "BENCH FAILED"; tail -20 gpurun_out/r2_bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --gpus 2 --share-device --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2_bench_share2.json 2> gpurun_out/r2_bench_share2.err || { echo "SHARE2 FAILED"; tail -20 gpurun_out/r2_bench_share2.err; exit 1; }
python bench.py --gpus 2 --steps 1 > gpurun_out/r2_bench_gpus2_refuse.txt 2>&1; echo "gpus2 rc=$?"
