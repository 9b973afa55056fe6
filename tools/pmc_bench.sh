#!/bin/bash
# HBM traffic of the bench's kernels: two separate PMC passes (FETCH_SIZE, WRITE_SIZE; kernel
# trace only) over short eager bench runs, one pair per workload and rays per rank.
# Summarised by tools/traffic_summary.py.
#     bash tools/pmc_bench.sh c4:4096 c4:512 c5:32768
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_bench
mkdir -p $OUT
for run in "$@"; do
  cfg=${run%%:*}; rays=${run##*:}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/${cfg}_rays${rays}_$ctr -o p -- python3 bench.py --config $cfg --global-batch $rays --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/${cfg}_rays${rays}_$ctr.log 2>&1
    rc=$?
    echo "$run $ctr rc=$rc" >> $OUT/summary.txt
    if [ $rc -ne 0 ]; then tail -20 $OUT/${cfg}_rays${rays}_$ctr.log; exit $rc; fi
  done
done
