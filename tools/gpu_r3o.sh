# round 3 (session 3): packed sine-epilogue arithmetic A/B (SPN_PK_EPI 0 build vs default), C5 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
CONFIG=c5 bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_nopk.so" "trunk2=3" "lib=libspnerf_amd_nopk.so" "trunk2=3"
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_nopk.so" "trunk2=0" "lib=libspnerf_amd_nopk.so" "trunk2=0"
