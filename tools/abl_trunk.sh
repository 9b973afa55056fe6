# Training-trunk variants on the current tree (ablation build for the non-product ones), C4 and
# C4@512, one call: 128-point tiles (product), 64-point tiles with the register-D epilogue (product
# option trunk_tile=64), 64-point tiles with the D image (ablation build: trunk_dreg=0).
cd $GRAFT_REPO_ROOT
for r in 1 2; do
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_abl.so" "lib=libspnerf_amd_abl.so trunk_tile=64" "lib=libspnerf_amd_abl.so trunk_tile=64 trunk_dreg=0"
EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_abl.so" "lib=libspnerf_amd_abl.so trunk_tile=64" "lib=libspnerf_amd_abl.so trunk_tile=64 trunk_dreg=0"
done
