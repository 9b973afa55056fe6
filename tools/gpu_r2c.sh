# GPU-box: fused-trunk tests, per-call trunk timings, C3/C5 benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_trunk.py > gpurun_out/t_trunk.txt 2>&1; rc=$?
tail -1 gpurun_out/t_trunk.txt; grep -E "FAILED|Error" gpurun_out/t_trunk.txt | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/trunk_bench.py > gpurun_out/tb.txt 2>&1 || { cat gpurun_out/tb.txt; exit 1; }
cat gpurun_out/tb.txt
for spec in "c3|" "c5|"; do
  cfg=${spec%%|*}; opt=${spec#*|}
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline $opt > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench $spec failed"; tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$spec',round(d['value']),round(d['ms_per_step'],3),d['roofline']['kernel'][:14],round(d['roofline']['achieved'],1),{k:(v['launches'],round(v['ms_per_step'],3)) for k,v in d.get('kernels',{}).items() if 'gemm' in k or 'trunk' in k})"
done
exit 0
