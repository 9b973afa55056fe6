# GPU-box: tests, C3 bench, rocprofv3 kernel-trace stats of the C3 and C2 benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print('c3',d['value'],d['ms_per_step'],d['roofline']['achieved'],d['mlp_gemms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof c3 failed"; tail -20 gpurun_out/prof_c3.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || { echo "rocprof c2 failed"; tail -20 gpurun_out/prof_c2.log; exit 1; }
ls -R gpurun_out/prof_c3 | head
exit 0
