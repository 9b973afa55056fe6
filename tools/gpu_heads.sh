# GPU-box: full GPU suite, then output-head A/B (heads_variant 0 / 1 / 2) per forward call and C5 / C3 benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
for v in ${HEADS_VARIANTS:-0 1 2}; do
  timeout -k 10 300 python tools/trunk_bench.py --rays 8192 --samples 128 --option heads_variant=$v > gpurun_out/heads_v$v.txt 2>&1 || { tail -20 gpurun_out/heads_v$v.txt; exit 1; }
  echo "heads_variant=$v"; grep -v amdgpu.ids gpurun_out/heads_v$v.txt | sed -e "s/'trunk_bf16.*'heads_fwd'/'heads_fwd'/"
done
for cfg in c5 c3; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg',round(d['value']),round(d['ms_per_step'],3))"
done
