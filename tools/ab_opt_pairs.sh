# The bench line under library options, alternating, REPS rounds (default 2), in one call:
#   bash tools/ab_opt_pairs.sh "opt=a" "opt=b"   (CONFIG, EXTRA as in gpu_ab_opt.sh)
cd $GRAFT_REPO_ROOT
for r in $(seq ${REPS:-2}); do bash tools/gpu_ab_opt.sh "$@" || exit 1; done
