# round 3 (session 3): packed epilogue arithmetic in the training / two-workgroup trunks — bitwise tests, C4 and C5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py tests/test_gpu_c5.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3n_tests.log | head -20; tail -5 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
bash tools/gpu_ab_opt.sh "trunk_dreg=1" "trunk_dreg=1"
CONFIG=c5 bash tools/gpu_ab_opt.sh "trunk2=3" "trunk2=3"
