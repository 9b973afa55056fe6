# GPU-box: fp32 TN point-split sweep at K = 512 and K = 64 (layer 0), P = 65 536 (C2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_bench 65536 512 > gpurun_out/tnsweep_512.txt 2>&1 || { tail -5 gpurun_out/tnsweep_512.txt; exit 1; }
timeout -k 10 120 ./tools/gemm_bench 65536 64 > gpurun_out/tnsweep_64.txt 2>&1 || { tail -5 gpurun_out/tnsweep_64.txt; exit 1; }
grep -E "tn " gpurun_out/tnsweep_512.txt gpurun_out/tnsweep_64.txt
