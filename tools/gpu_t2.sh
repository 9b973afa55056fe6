set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trunk.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t2_test.log 2>&1; rc=$?
tail -15 gpurun_out/t2_test.log
[ $rc -eq 0 ] || exit 1
CONFIG=c4 timeout -k 10 400 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=1" "trunk2=0" "trunk2=1"
CONFIG=c5 timeout -k 10 300 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=2"
