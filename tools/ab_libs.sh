# A/B of in-tree library builds in one call: gradient / render hashes of one C4 step at 4096 and 512
# rays under each (equal = bit-identical), then the C4 and C4@512 bench lines alternating, REPS rounds.
#     LIBS="libspnerf_amd_prev.so libspnerf_amd_x.so libspnerf_amd.so" bash tools/ab_libs.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in $LIBS; do
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py 2>/dev/null || exit 1
  SPNERF_AMD_LIB=$lib timeout -k 10 120 python tools/grad_hash.py --global-batch 512 2>/dev/null || exit 1
done
args=""; for lib in $LIBS; do args="$args lib=$lib"; done
for r in $(seq ${REPS:-2}); do
  bash tools/gpu_ab_opt.sh $args || exit 1
  EXTRA="--global-batch 512" bash tools/gpu_ab_opt.sh $args || exit 1
done
