# GPU-box: fp32 NT variants (microbench incl. bit-equality vs variant 0), then the C2 bench at
# nt_f32_variant 6 and 7 (same k-order: the final losses must be equal).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/gemm_bench 65536 512 > gpurun_out/gb32.txt 2>&1 || { cat gpurun_out/gb32.txt; exit 1; }
cat gpurun_out/gb32.txt
for v in ${VS:-6 7 6 7}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --option nt_f32_variant=$v > gpurun_out/b_nt$v.json 2> gpurun_out/b_nt$v.err || { tail -20 gpurun_out/b_nt$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_nt$v.json'));print('nt$v',round(d['value']),round(d['ms_per_step'],3),round(d['roofline']['achieved'],1),d['final_loss'])"
done
