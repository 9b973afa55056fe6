# GPU-box: GPU suite + C3 / C5 benches (graph mode default).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
for cfg in c3 c5; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg',round(d['value']),round(d['ms_per_step'],3),'nt',round(d['roofline']['achieved'],1),'gemms',round(d['mlp_gemms']['frac'],3))"
done
