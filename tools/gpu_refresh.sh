# GPU-box, end-of-round refresh: full suite + smoke + C2/C3/C5 benches + rocprof stats
# (tools/gpu_full.sh), then the PMC traffic passes (tools/pmc_bench.sh) and the PMC clock pass.
set -o pipefail
bash tools/gpu_full.sh || exit $?
bash tools/pmc_bench.sh || exit $?
bash tools/pmc_clock.sh > gpurun_out/pmc_clock_summary.txt 2>&1 || { cat gpurun_out/pmc_clock_summary.txt; exit 1; }
echo refresh done
