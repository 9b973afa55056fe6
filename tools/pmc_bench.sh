#!/bin/bash
# HBM traffic of the bench's kernels: two separate PMC passes (FETCH_SIZE, WRITE_SIZE; kernel
# trace only) over short eager bench runs.  Summarised by tools/traffic_summary.py.
#     bash tools/pmc_bench.sh c4 c5
set -u
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_bench
mkdir -p $OUT
for cfg in "$@"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/${cfg}_$ctr -o p -- python3 bench.py --config $cfg --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/${cfg}_$ctr.log 2>&1
    rc=$?
    echo "$cfg $ctr rc=$rc" >> $OUT/summary.txt
    if [ $rc -ne 0 ]; then tail -20 $OUT/${cfg}_$ctr.log; exit $rc; fi
  done
done
