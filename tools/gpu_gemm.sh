# GPU-box: bf16 GEMM microbench only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/gemm_bench_bf16 > gpurun_out/gb16.txt 2>&1; rc=$?
cat gpurun_out/gb16.txt
exit $rc
