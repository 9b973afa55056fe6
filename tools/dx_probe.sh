# The dX chain's extra reads: FETCH_SIZE / L2 hits and misses of the C4 step's
# kernels under ablation options, then the bench line with non-temporal D loads against the default.
cd $GRAFT_REPO_ROOT
bash tools/pmc_dx.sh "" "trunk_bwd_nt=2" "trunk_dbg=2" "trunk_dbg=1" &&
CTR="TCC_HIT_sum TCC_MISS_sum" bash tools/pmc_dx.sh "" "trunk_bwd_nt=2" &&
for r in 1 2; do bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_abl.so" "lib=libspnerf_amd_abl.so trunk_bwd_nt=2"; done
