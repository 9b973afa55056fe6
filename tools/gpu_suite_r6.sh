# smoke + the whole -m gpu suite (one process), then the default bench line exactly as the driver
# runs it.  Usage: bash tools/gpu_suite_r6.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-suite}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 500 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/$T/gputest.log | head -20; tail -20 gpurun_out/$T/gputest.log; exit 1; }
tail -1 gpurun_out/$T/gputest.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { echo "BENCH FAILED"; tail -20 gpurun_out/$T/bench_default.err; exit 1; }
wc -c gpurun_out/$T/bench_default.json
python -c "import json; d=json.load(open('gpurun_out/$T/bench_default.json')); print('C4', d['ms_per_step'], d['value'], d['roofline']['frac'], d['mlp_mfma_utilisation']['frac'], 'C2', d['secondary']['c2']['ms_per_step'], 'C5', d['secondary']['c5']['ms_per_step'], d['secondary']['c5']['roofline']['frac'])"
