# GPU-box: GEMM microbenches (fp32 + bf16)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/gemm_bench 65536 512 > gpurun_out/gb32.txt 2>&1; rc=$?
cat gpurun_out/gb32.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 ./tools/gemm_bench_bf16 > gpurun_out/gb16.txt 2>&1; rc=$?
grep -E "131072|variant|checks|FAIL" gpurun_out/gb16.txt
exit $rc
