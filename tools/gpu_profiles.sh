# Round profiles: PMC traffic of C4 / C5, then rocprofv3 kernel stats of the default bench command
# and of the C5 bench.  Outputs under gpurun_out/ (copied to profiles/<round>/ by hand).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc_bench.sh c4:4096 c4:512 c5:32768 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o p -- python3 bench.py > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err || { tail gpurun_out/prof_default.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o p -- python3 bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err || { tail gpurun_out/prof_c5.err; exit 1; }
echo done
