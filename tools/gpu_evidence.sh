# Round-end evidence of the committed tree: smoke(), the -m gpu suite, the bench lines (default C4
# with the CPU baseline and the long PSNR study, C4 at 512 rays, C3, C5), then PMC traffic and
# rocprofv3 kernel stats (tools/gpu_profiles.sh).  Usage: bash tools/gpu_evidence.sh TAG [noprof]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-evidence}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/$T/gputest.log | head -20; tail -20 gpurun_out/$T/gputest.log; exit 1; }
tail -1 gpurun_out/$T/gputest.log
timeout -k 10 700 python -u bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { echo "BENCH FAILED"; tail -20 gpurun_out/$T/bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --config c4 --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c4_512.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c3.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c5.json 2>/dev/null || exit 1
for f in default c4_512 c3 c5; do python -c "import json; d=json.load(open('gpurun_out/$T/bench_$f.json')); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,2), d['roofline']['kernel'][:22], round(d['roofline']['frac'],3), (d.get('mlp_mfma_utilisation') or {}).get('frac'))"; done
[ "${2:-}" = "noprof" ] || bash tools/gpu_profiles.sh
