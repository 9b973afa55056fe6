# round 3 (session 3): C4 step with the two-workgroup training trunk (non-temporal H copy-outs) vs the default
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_opt.sh "trunk2=3" "trunk2=2 trunk2_tile=64" "trunk2=1 trunk2_tile=64" "trunk2=3" "trunk2=2 trunk2_tile=64" "trunk2=1 trunk2_tile=64"
GB=512 bash tools/ab512.sh "trunk2=3" "trunk2=2 trunk2_tile=64" "trunk2=3" "trunk2=2 trunk2_tile=64"
