# GPU check of the whole tree: the -m gpu suite, then the default bench line (C4 + C2 beside it).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAILED|Error|error" gpurun_out/${TAG}_gputest.log | head -20; tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
if [ "${2:-bench}" = "bench" ]; then
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('C4', d['ms_per_step'], d['value'], 'C2', d['secondary']['c2']['ms_per_step'])"
timeout -k 10 300 python3 bench.py --config c4 --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/${TAG}_c4_512.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/${TAG}_c4_512.json')); print('C4@512', d['ms_per_step'], d['value'])"
fi
