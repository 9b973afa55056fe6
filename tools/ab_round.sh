# Round-over-round A/B in one call: the start-of-round build (libspnerf_amd_r5.so) against the
# current tree on C5, C4 and C4@512, alternating, two rounds; gradient hashes of both first.
cd $GRAFT_REPO_ROOT
for lib in libspnerf_amd.so libspnerf_amd_r5.so; do
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py 2>/dev/null || exit 1
done
for r in 1 2; do
CONFIG=c5 bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_r5.so" "lib=libspnerf_amd.so"
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_r5.so" "lib=libspnerf_amd.so"
EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_r5.so" "lib=libspnerf_amd.so"
done
