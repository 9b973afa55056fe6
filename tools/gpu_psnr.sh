# GPU-box: PSNR-parity test and the default bench line (with cpu_baseline + psnr_parity)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_psnr.py tests/test_gpu_trunk.py > gpurun_out/t_psnr.txt 2>&1; rc=$?
grep -E "psnr|bitwise|passed|failed|Error" gpurun_out/t_psnr.txt | head -20
[ $rc -ne 0 ] && { tail -30 gpurun_out/t_psnr.txt; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value'],d['ms_per_step'],d['cpu_baseline']['value'],d['psnr_parity'])"
