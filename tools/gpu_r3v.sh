# round 3 (session 3): non-temporal H copy-outs as the default — tests, A/B pairs at 4096 / 512 rays, C3, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py tests/test_gpu_bf16.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3v_tests.log | head -20; tail -5 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
GB=512 bash tools/ab512.sh "trunk_nt=0" "trunk_nt=1" "trunk_nt=0" "trunk_nt=1"
bash tools/gpu_ab_opt.sh "trunk_nt=0" "trunk_nt=1" "trunk_nt=0" "trunk_nt=1"
CONFIG=c3 bash tools/gpu_ab_opt.sh "trunk_nt=0" "trunk_nt=1"
CONFIG=c5 bash tools/gpu_ab_opt.sh "trunk_nt=0" "trunk_nt=1"
