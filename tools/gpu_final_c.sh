# end of round 3: smoke() and the -m gpu suite on the committed tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final4
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final4/smoke.log 2>&1 || { tail -20 gpurun_out/final4/smoke.log; exit 1; }
tail -1 gpurun_out/final4/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final4/gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/final4/gputest.log | head -20; tail -20 gpurun_out/final4/gputest.log; exit 1; }
tail -1 gpurun_out/final4/gputest.log
