#!/bin/bash
# Where the dX chain's extra HBM reads come from: FETCH_SIZE (one pass each, kernel trace only) of
# the C4 step's kernels under library options of the ablation build, per-launch means by class.
#     bash tools/pmc_dx.sh "" "trunk_bwd_nt=2" "trunk_bwd_dbg=2" ...   (summary: gpurun_out/pmc_dx/summary.txt)
# Options run on libspnerf_amd_abl.so (make variant VDEF=-DSPN_ABLATIONS VLIB=libspnerf_amd_abl.so).
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_dx
mkdir -p $OUT
n=0
for o in "$@"; do
  n=$((n + 1))
  args=""; for kv in $o; do args="$args --option $kv"; done
  SPNERF_AMD_LIB=${LIB:-libspnerf_amd_abl.so} timeout -s KILL 300 rocprofv3 --pmc ${CTR:-FETCH_SIZE} --kernel-trace --output-format csv \
    -d $OUT/run$n -o p -- python3 bench.py --config c4 --global-batch ${GB:-4096} --eager --steps 2 --warmup 1 \
    --no-cpu-baseline --no-secondary $args > $OUT/run$n.log 2>&1 || { tail -20 $OUT/run$n.log; exit 1; }
  echo "[$o] $(python3 tools/pmc_dx_summary.py $OUT/run$n)" | tee -a $OUT/summary.txt
done
