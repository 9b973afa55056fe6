set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_reuse.py} -x -v --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/t.log | tail -25; tail -1 gpurun_out/t.log; exit $rc
