# round 3 (session 3): non-temporal dZ stores / D loads in the fused dX chain, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
GB=512 bash tools/ab512.sh "trunk_bwd_nt=0" "trunk_bwd_nt=1" "trunk_bwd_nt=2" "trunk_bwd_nt=3" "trunk_bwd_nt=0" "trunk_bwd_nt=3"
bash tools/gpu_ab_opt.sh "trunk_bwd_nt=0" "trunk_bwd_nt=1" "trunk_bwd_nt=2" "trunk_bwd_nt=3" "trunk_bwd_nt=0" "trunk_bwd_nt=3"
