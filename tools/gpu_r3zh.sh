# round 3 (session 3): what the training trunk's epilogue costs (ablations, outputs invalid)
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in "trunk_var=0" "trunk_var=32" "trunk_var=256" "trunk_dbg=1" "trunk_var=256 trunk_dbg=1" "trunk_var=0"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
