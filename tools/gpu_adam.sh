# GPU-box: Adam test + ABI test, then C2 with the library Adam and with torch's fused Adam.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_adam.py tests/test_abi.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/adam.txt 2>&1; rc=$?
tail -3 gpurun_out/adam.txt; [ $rc -ne 0 ] && exit $rc
for o in "" "--torch-adam" "" "--torch-adam"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $o > gpurun_out/b_adam.json 2> gpurun_out/b_adam.err || { tail -20 gpurun_out/b_adam.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_adam.json'));print('adam[$o]',round(d['value']),round(d['ms_per_step'],3),d['final_loss'])"
done
