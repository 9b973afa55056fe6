# The whole -m gpu suite and smoke() in one call (no bench): bash tools/gpu_quick.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-quick}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 500 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/$T/gputest.log | head -20; tail -30 gpurun_out/$T/gputest.log; exit 1; }
grep -E "difference|bf16 outputs" gpurun_out/$T/gputest.log | tail -8
tail -1 gpurun_out/$T/gputest.log
