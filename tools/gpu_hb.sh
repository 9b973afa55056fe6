# GPU-box: full GPU suite, then C3 and C2 benches (heads_bwd timing).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
for cfg in c3 c2; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/b_hb_$cfg.json 2> gpurun_out/b_hb_$cfg.err || { tail -20 gpurun_out/b_hb_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_hb_$cfg.json'));k=d['kernels'];print('$cfg',round(d['value']),round(d['ms_per_step'],3),'heads_bwd',round(k['heads_bwd']['ms_per_step'],3),'heads_fwd',round(k['heads_fwd']['ms_per_step'],3))"
done
