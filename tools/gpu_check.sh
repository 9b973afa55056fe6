# GPU-box check: GPU test suite (fp32 parity + bf16), benches (c3 bf16, c2 fp32).  Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -s > gpurun_out/gpu_tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.txt | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print('c3',d['value'],d['ms_per_step'],d['roofline'],d['mlp_gemms'])"
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'])"
exit $rc
