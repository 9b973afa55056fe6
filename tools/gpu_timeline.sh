# rocprofv3 kernel trace of short C4 bench runs (graph mode) at the given global batches;
# tools/timeline.py prints the last steps of each (busy, idle gaps, sequence).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-tl}
shift
for gb in "$@"; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$gb -o t -- python3 bench.py --config c4 --global-batch $gb --steps 3 --warmup 2 --prof-steps 1 --no-cpu-baseline --no-secondary > gpurun_out/${TAG}_$gb.log 2>&1 || { tail gpurun_out/${TAG}_$gb.log; exit 1; }
done
