# GPU-box check: bf16 tests, full GPU suite, benches (c3 bf16, c2 fp32).  Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_bf16.py -q -s -p no:cacheprovider > gpurun_out/bf16_tests.txt 2>&1; rc=$?
grep -E "^(c1|c3|beta|nomap|rgb|depth|sem|sun|worst|\{)|passed|failed" gpurun_out/bf16_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
exit $rc
