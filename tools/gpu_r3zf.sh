# round 3 (session 3): tn_bf16_ip 1 vs 2 (the default), pairs at 4096 and 512 rays
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_opt.sh "tn_bf16_ip=2" "tn_bf16_ip=1" "tn_bf16_ip=2" "tn_bf16_ip=1" "tn_bf16_ip=2" "tn_bf16_ip=1"
GB=512 bash tools/ab512.sh "tn_bf16_ip=2" "tn_bf16_ip=1" "tn_bf16_ip=2" "tn_bf16_ip=1"
