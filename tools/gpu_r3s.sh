# round 3 (session 3): which of the training trunk's HBM writes costs (ablations, outputs invalid)
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in "trunk_dbg=0" "trunk_dbg=4" "trunk_dbg=8" "trunk_dbg=1" "trunk_dbg=0"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
