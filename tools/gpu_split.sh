# GPU-box: TN split-cap change — GPU suite, microbench (bf16 TN), C2 and C3 benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 120 ./tools/gemm_bench_bf16 131072 20 tn 2 > gpurun_out/tn16_micro.txt 2>&1 || { cat gpurun_out/tn16_micro.txt; exit 1; }
grep -E "P=131072|checks" gpurun_out/tn16_micro.txt
for cfg in c2 c3; do
timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/$cfg.json 2> gpurun_out/$cfg.err || { tail -20 gpurun_out/$cfg.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$cfg.json'));k=d['kernels'];print('$cfg',round(d['value']),round(d['ms_per_step'],3),{n:(k[n]['launches'],round(k[n]['avg_us'],1),round(k[n]['ms_per_step'],3)) for n in k if 'gemm' in n})"
done
