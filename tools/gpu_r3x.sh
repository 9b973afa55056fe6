# round 3 (session 3): non-temporal stores of the DMA NT GEMM (SPN_NT16_NT=1 build), A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
GB=512 bash tools/ab512.sh "trunk_nt=1" "lib=libspnerf_amd_ntnt.so" "trunk_nt=1" "lib=libspnerf_amd_ntnt.so"
bash tools/gpu_ab_opt.sh "trunk_nt=1" "lib=libspnerf_amd_ntnt.so" "trunk_nt=1" "lib=libspnerf_amd_ntnt.so"
