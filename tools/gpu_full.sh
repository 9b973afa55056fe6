# GPU-box: full GPU suite, smoke, default bench (with CPU baseline), rocprof of C2 / C3 benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof c3 failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || { echo "rocprof c2 failed"; tail -20 gpurun_out/prof_c2.log; exit 1; }
grep -E "^\{" gpurun_out/prof_c2.log | python -c "import sys,json;d=json.loads(sys.stdin.read());print('c2 under rocprof', d['value'], d['roofline']['avg_launch_us'])"
exit 0
