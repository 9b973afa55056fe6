# GPU-box: TN variants (microbench, bit-equality of the slabs), then C2 at tn_f32_variant 1 / 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/gemm_bench 65536 512 > gpurun_out/gb32.txt 2>&1 || { cat gpurun_out/gb32.txt; exit 1; }
grep -E "tn|variant 8" gpurun_out/gb32.txt
for v in 1 2 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --option tn_f32_variant=$v > gpurun_out/b_tn$v.json 2> gpurun_out/b_tn$v.err || { tail -20 gpurun_out/b_tn$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_tn$v.json'));k=d['kernels'];print('tn$v',round(d['value']),round(d['ms_per_step'],3),'tn',round(k['gemm_tn_f32']['ms_per_step'],3),round(k['gemm_tn_f32']['tflops'],1),d['final_loss'])"
done
