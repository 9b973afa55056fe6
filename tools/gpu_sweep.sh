set -o pipefail
cd $GRAFT_REPO_ROOT
EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh "" "trunk_tile=64" "defer_heads=1" "defer_heads=0" "tn_group=5" "" "trunk_tile=64" || exit 1
bash tools/gpu_ab_opt.sh "" "trunk_tile=64" "defer_heads=1" "" "trunk_tile=64" || exit 1
