#!/bin/bash
# PMC passes over tools/gemm_bench_bf16 (one counter group per pass, kernel-trace only).
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc16
mkdir -p $OUT
i=0
for grp in "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- ./tools/gemm_bench_bf16 131072 2 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc" >> $OUT/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
