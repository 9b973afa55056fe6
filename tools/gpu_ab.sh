# GPU-box: full GPU suite, then an A/B of one library option per MLP forward call
# (OPT=name VALS="0 1"), then the C5 / C3 benches at the defaults.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
for v in $VALS; do
  timeout -k 10 300 python tools/trunk_bench.py --rays 8192 --samples 128 --option $OPT=$v > gpurun_out/ab_$v.txt 2>&1 || { tail -20 gpurun_out/ab_$v.txt; exit 1; }
  echo "$OPT=$v"; grep -v amdgpu.ids gpurun_out/ab_$v.txt
done
for cfg in c5 c3; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg',round(d['value']),round(d['ms_per_step'],3))"
done
