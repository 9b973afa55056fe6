# GPU-box: full GPU suite, C2 bench twice, rocprof stats of the C2 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gpu_tests.txt | head; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_red$i.json 2> gpurun_out/b_red$i.err || { tail -20 gpurun_out/b_red$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_red$i.json'));print('c2',round(d['value']),round(d['ms_per_step'],3),round(d['roofline']['achieved'],1),d['final_loss'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
grep -E "reduce_slabs|k_gemm_nt_w|k_gemm_tn" gpurun_out/prof_c2/c2_kernel_stats.csv | cut -d, -f1-4
