# GPU-box: benches in graph (default) and eager mode.
set -o pipefail
mkdir -p gpurun_out
for cfg in c3 c2; do
  for mode in graph eager; do
    flag=""; [ $mode = eager ] && flag="--eager"
    timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline $flag > gpurun_out/bench_${cfg}_$mode.json 2> gpurun_out/bench_${cfg}_$mode.err || { echo "bench $cfg $mode failed"; tail -20 gpurun_out/bench_${cfg}_$mode.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_${cfg}_$mode.json'));print('$cfg $mode',round(d['value']),round(d['ms_per_step'],3),round(d['roofline']['achieved'],1),d['execution'][:40])"
    grep -i "capture" gpurun_out/bench_${cfg}_$mode.err || true
  done
done
