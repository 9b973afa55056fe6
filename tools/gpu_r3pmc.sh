# round 3 (session 3): clock / MFMA busy / VALU / LDS / wait counters of the C4 step's kernels (two PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c4 bash tools/pmc_clock.sh > gpurun_out/pmc_c4_final.txt 2>&1 || { tail -20 gpurun_out/pmc_c4_final.txt; exit 1; }
cat gpurun_out/pmc_c4_final.txt | head -60
