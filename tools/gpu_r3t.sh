# round 3 (session 3): non-temporal copy-outs of the register-D training trunk
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in "trunk_nt=0" "trunk_nt=1" "trunk_nt=4" "trunk_nt=5" "trunk_nt=0" "trunk_nt=5"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
bash tools/gpu_ab_opt.sh "trunk_nt=0" "trunk_nt=5" "trunk_nt=0" "trunk_nt=5"
