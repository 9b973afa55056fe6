# round 3 (session 3): training-trunk ablations with D from the registers + PMC waits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in "trunk_dreg=0" "trunk_dreg=1" "trunk_dreg=1 trunk_dbg=1" "trunk_dreg=0 trunk_dbg=1"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
OUT=$PWD/gpurun_out/pmc_r3m
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/p1 -o p -- python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 3 --option trunk_dreg=1 > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $OUT/p2 -o p -- python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 3 --option trunk_dreg=1 > $OUT/p2.log 2>&1 || { tail $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT | grep -B1 -A1 trunk
