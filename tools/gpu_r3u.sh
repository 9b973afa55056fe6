# round 3 (session 3): layer 0 inside the training trunk (trunk_l0 2) and non-temporal H copy-outs, C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_opt.sh "trunk_l0=1" "trunk_l0=2" "trunk_nt=1" "trunk_l0=1" "trunk_l0=2" "trunk_nt=1"
GB=512 bash tools/ab512.sh "trunk_l0=1" "trunk_l0=2" "trunk_nt=1"
