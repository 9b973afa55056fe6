# round 3 (session 3): fused dX chain with dZ stored from the registers — bitwise tests, A/B pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_trunk.py -x -v --timeout 200 --timeout-method thread -k "backward or trunk or rowsum" > gpurun_out/r3p_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3p_tests.log | head -20; tail -5 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
bash tools/gpu_ab_opt.sh "trunk_bwd_dreg=0" "trunk_bwd_dreg=1" "trunk_bwd_dreg=0" "trunk_bwd_dreg=1"
GB=512 bash tools/ab512.sh "trunk_bwd_dreg=0" "trunk_bwd_dreg=1"
