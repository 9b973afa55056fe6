#!/bin/bash
# Effective clock, MFMA-pipe occupancy, wait states and LDS bank conflicts of the C4 training
# step's kernels (tools/pmc_clock.sh's two SQ + GRBM passes, kernel trace only) over a short eager
# C4 run at GB rays (default 4096), no CPU leg or secondary lines.  Summarised by
# tools/pmc_summary.py into gpurun_out/pmc_c4/summary.txt.
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_c4
mkdir -p $OUT
ARGS="--config c4 --global-batch ${GB:-4096} --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o p -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/p2 -o p -- python3 bench.py $ARGS > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
