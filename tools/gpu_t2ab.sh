# trunk2 tilings: GPU tests, per-call timings of the training forward at C4 size, C4 / C5 lines
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trunk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2ab_tests.log 2>&1 || { tail -30 gpurun_out/t2ab_tests.log; exit 1; }
tail -2 gpurun_out/t2ab_tests.log
for o in "trunk2=0" "trunk2=1 trunk2_tile=128" "trunk2=1 trunk2_tile=64" "trunk2=1 trunk2_tile=128 trunk_dbg=3"; do
args=""; for kv in $o; do args="$args --option $kv"; done
echo "[$o]"; timeout -k 10 120 python tools/trunk_bench.py --rays 4096 --samples 128 --modes save,nosave $args 2>&1 | grep -v amdgpu.ids | grep -v resident || exit 1
done
CONFIG=c4 timeout -k 10 400 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=1 trunk2_tile=128" "trunk2=1 trunk2_tile=64"
CONFIG=c5 timeout -k 10 300 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=2 trunk2_tile=128"
