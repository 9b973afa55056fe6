# GPU-box: bf16 TN microbench (checks + timings of the three tilings), variants tests, C3 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_bench_bf16 131072 20 tn 0 > gpurun_out/tn16_micro.txt 2>&1 || { cat gpurun_out/tn16_micro.txt; exit 1; }
grep -E "P=131072|checks" gpurun_out/tn16_micro.txt
bash tools/gpu_tn16.sh
