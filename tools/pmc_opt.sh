#!/bin/bash
# SQ / GRBM counters (clock, MFMA busy, waits, LDS conflicts) of the C4 step's kernels under library
# options: OPTS="--option tn_bf16_m16=1" bash tools/pmc_opt.sh TAG  (summary: gpurun_out/pmc_TAG/summary.txt)
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_$1
mkdir -p $OUT
ARGS="--config c4 --global-batch ${GB:-4096} --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary ${OPTS:-}"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o p -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/p2 -o p -- python3 bench.py $ARGS > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && grep -A1 "gemm_tn" $OUT/summary.txt
