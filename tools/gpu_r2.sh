# GPU-box: fused-trunk + wide fp32 GEMM checks, then A/B benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_trunk.py tests/test_gpu_bf16.py > gpurun_out/t_trunk.txt 2>&1; rc=$?
tail -3 gpurun_out/t_trunk.txt; grep -E "bitwise|FAILED|Error" gpurun_out/t_trunk.txt | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./tools/gemm_bench 65536 512 > gpurun_out/gb32.txt 2>&1 || { cat gpurun_out/gb32.txt; exit 1; }
cat gpurun_out/gb32.txt
for spec in "c3|" "c3|--option fused_trunk=0" "c2|" "c2|--option nt_f32_variant=4" "c2|--option nt_f32_variant=5"; do
  cfg=${spec%%|*}; opt=${spec#*|}
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline $opt > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench $spec failed"; tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$spec',round(d['value']),round(d['ms_per_step'],3),d['roofline']['kernel'][:14],round(d['roofline']['achieved'],1),{k:(v['launches'],round(v['ms_per_step'],3)) for k,v in d['kernels'].items() if 'gemm' in k or 'trunk' in k})"
done
exit 0
