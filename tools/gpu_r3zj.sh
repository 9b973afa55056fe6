# round 3 (session 3): register-D epilogue without the per-feature-tile scheduling fence (SPN_EPI_FENCE 0 build), A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libspnerf_amd_nofence.so libspnerf_amd.so libspnerf_amd_nofence.so libspnerf_amd.so; do
echo "== $lib"; SPNERF_AMD_LIB=$lib timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 --option trunk_var=0 2>&1 | grep save || exit 1
done
