# A/B of the working tree's library against sp-nerf_amd/libspnerf_amd_prev.so (the previous
# commit's build): gradient / render hashes of one C4 step at 4096 and 512 rays under both (equal =
# bit-identical), then the C4 and C4@512 bench lines alternating, REPS rounds, in one call.
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libspnerf_amd.so libspnerf_amd_prev.so; do
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py 2>/dev/null || exit 1
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py --global-batch 512 2>/dev/null || exit 1
done
for r in $(seq ${REPS:-2}); do
  bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so" || exit 1
  EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so" || exit 1
done
