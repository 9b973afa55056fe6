#!/bin/bash
# Effective clock and MFMA-pipe occupancy of the C2 bench's GEMMs: one PMC pass (SQ + GRBM
# counters, kernel trace only) over a short eager C2 run.  Summarised by tools/pmc_summary.py.
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_clock
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o p -- python3 bench.py --config ${CFG:-c2} --eager --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p1.log 2>&1
rc=$?
[ $rc -ne 0 ] && tail -20 $OUT/p1.log && exit $rc
# second pass: LDS bank conflicts and wait states
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/p2 -o p -- python3 bench.py --config ${CFG:-c2} --eager --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p2.log 2>&1
rc=$?
[ $rc -ne 0 ] && tail -20 $OUT/p2.log
python3 tools/pmc_summary.py $OUT
exit $rc
