# round 3 (session 3): DMA issue placement of the weight-gradient / NT GEMMs re-measured on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_opt.sh "tn_bf16_ip=2" "tn_bf16_ip=0" "tn_bf16_ip=1" "tn_bf16_ip=2" "nt_bf16_ip=0" "nt_bf16_ip=1" "nt_bf16_ip_gen=0" "tn_bf16_ip=2"
