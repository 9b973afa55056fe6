# GPU-box: bf16 TN tilings — variants test, then C3 bench with each tiling.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_variants.py -k bf16 tests/test_gpu_bf16.py > gpurun_out/tn16_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/tn16_tests.txt
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/tn16_tests.txt | head -20; exit $rc; }
for v in 2 3; do
  timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --option tn_bf16_variant=$v > gpurun_out/c3_tn$v.json 2> gpurun_out/c3_tn$v.err || { tail -20 gpurun_out/c3_tn$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c3_tn$v.json'));k=d['kernels'];print('tn$v',round(d['value']),round(d['ms_per_step'],3),{n:(k[n]['launches'],round(k[n]['avg_us'],1),round(k[n]['ms_per_step'],3)) for n in k if 'tn' in n or 'reduce' in n})"
done
