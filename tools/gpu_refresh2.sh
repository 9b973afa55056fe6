# GPU-box: full suite + smoke + C2/C3/C5 benches + rocprof stats, then the PMC clock pass.
set -o pipefail
bash tools/gpu_full.sh || exit $?
bash tools/pmc_clock.sh > gpurun_out/pmc_clock_summary.txt 2>&1 || { cat gpurun_out/pmc_clock_summary.txt; exit 1; }
echo refresh done
