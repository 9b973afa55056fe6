# TN address precompute A/B: bit-identity (gradient hashes) and C4 / C4@512 lines, alternating
# libraries in one call.  Needs sp-nerf_amd/libspnerf_amd_prev.so (make variant VDEF=-DSPN_TN_ADDR=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libspnerf_amd.so libspnerf_amd_prev.so; do
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py 2>/dev/null || exit 1
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py --global-batch 512 2>/dev/null || exit 1
done
for r in 1 2; do
  bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so" || exit 1
  EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_prev.so" "lib=libspnerf_amd.so" || exit 1
done
