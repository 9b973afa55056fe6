#!/bin/bash
# PMC passes over tools/trunk_bench.py (training forward at C4 size) for the trunk tilings:
# effective clock, MFMA busy, VALU / MFMA / LDS instruction counts, waits, LDS bank conflicts.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for o in "trunk2=0" "trunk2=1 trunk2_tile=64" "trunk2=1 trunk2_tile=128"; do
tag=$(echo $o | tr ' =' '__')
args=""; for kv in $o; do args="$args --option $kv"; done
OUT=$PWD/gpurun_out/pmc_t2/$tag
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o p -- python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 3 $args > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/p2 -o p -- python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 3 $args > $OUT/p2.log 2>&1 || { tail $OUT/p2.log; exit 1; }
echo "== $o"; python3 tools/pmc_summary.py $OUT | grep -A1 trunk
done
