# round 3 (session 3): two-workgroup training trunk with non-temporal H copy-outs vs the one-workgroup default
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in "trunk2=3" "trunk2=1 trunk2_tile=64" "trunk2=1 trunk2_tile=64 trunk_nt=0" "trunk2=3"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
