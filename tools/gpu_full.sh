# GPU-box: full GPU suite, smoke, default bench (with CPU baseline), C3 / C5 benches, rocprof of
# the C2 / C3 / C5 benches (kernel trace + stats).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
for cfg in c3 c5; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg',round(d['value']),round(d['ms_per_step'],3),d['roofline']['kernel'][:14],round(d['roofline']['frac'],3))"
done
for spec in "c2|--steps 20 --warmup 5" "c3|--steps 10 --warmup 3" "c5|--steps 10 --warmup 3"; do
  cfg=${spec%%|*}; opt=${spec#*|}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o $cfg -- python3 bench.py --config $cfg $opt --no-cpu-baseline > gpurun_out/prof_$cfg.log 2>&1 || { echo "rocprof $cfg failed"; tail -20 gpurun_out/prof_$cfg.log; exit 1; }
done
exit 0
