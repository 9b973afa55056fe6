# GPU-box: parity + variants tests, then the default C2 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c2.json'));k=d['kernels'];print('c2',round(d['value']),round(d['ms_per_step'],3),{n:(k[n]['launches'],round(k[n]['avg_us'],1),round(k[n]['ms_per_step'],3)) for n in k if 'gemm' in n})"
