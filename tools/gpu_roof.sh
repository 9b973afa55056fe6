# GPU-box: bench roofline objects for C2 / C3 / C5 (short runs, no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
for cfg in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/roof_$cfg.json 2> gpurun_out/roof_$cfg.err || { tail -20 gpurun_out/roof_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/roof_$cfg.json'));print('$cfg',round(d['value']),json.dumps(d['roofline']))"
done
