# round 3 (session 3): 128-point training trunk tiles with D from the registers — bitwise tests, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_trunk.py -x -v --timeout 200 --timeout-method thread -k "register_d" > gpurun_out/r3q_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3q_tests.log | head -20; tail -5 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
for o in "trunk_tile=0" "trunk_tile=128" "trunk_tile=128 trunk_dreg=0"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "== $o"; timeout -k 10 120 python3 tools/trunk_bench.py --rays 4096 --samples 128 --modes save --iters 5 $args 2>&1 | grep save || exit 1
done
bash tools/gpu_ab_opt.sh "trunk_tile=0" "trunk_tile=128" "trunk_tile=0" "trunk_tile=128"
GB=512 bash tools/ab512.sh "trunk_tile=0" "trunk_tile=128"
