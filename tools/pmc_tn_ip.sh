#!/bin/bash
# HBM bytes of the weight-gradient GEMM under the two DMA issue points (ablation library: option
# tn_bf16_ip 1 = the four DMAs after the step's MFMAs, 3 = spread over them; the product runs 3):
# FETCH_SIZE and WRITE_SIZE passes over the same eager C4 line as tools/pmc_bench.sh.
set -u
export TMPDIR=/tmp SPNERF_AMD_LIB=libspnerf_amd_abl.so
OUT=$PWD/gpurun_out/pmc_tn_ip
mkdir -p $OUT
for ip in 1 3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/c4_rays4096_ip${ip}_$ctr -o p -- python3 bench.py --config c4 --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --option tn_bf16_ip=$ip > $OUT/ip${ip}_$ctr.log 2>&1
    rc=$?
    echo "ip $ip $ctr rc=$rc" >> $OUT/summary.txt
    if [ $rc -ne 0 ]; then tail -20 $OUT/ip${ip}_$ctr.log; exit $rc; fi
  done
done
