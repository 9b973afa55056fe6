# Round profiles: PMC traffic (C4 at 4096 and 512 rays per rank, C5), then rocprofv3 kernel stats of
# the default bench command (its long PSNR study off: --psnr-steps 0 keeps the trace bounded) and of
# the C5 bench.  Traces stay in /tmp; the stats CSVs and bench JSON land in gpurun_out/ (copied to
# profiles/<round>/ by hand).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash tools/pmc_bench.sh c4:4096 c4:512 c5:32768 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_default -o p -- python3 bench.py --psnr-steps 0 > gpurun_out/prof/default.json 2> gpurun_out/prof/default.err || { tail gpurun_out/prof/default.err; exit 1; }
cp $(find /tmp/prof_default -name "*kernel_stats.csv" -print -quit) gpurun_out/prof/c4_default_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c5 -o p -- python3 bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/prof/c5.json 2> gpurun_out/prof/c5.err || { tail gpurun_out/prof/c5.err; exit 1; }
cp $(find /tmp/prof_c5 -name "*kernel_stats.csv" -print -quit) gpurun_out/prof/c5_kernel_stats.csv
echo done
