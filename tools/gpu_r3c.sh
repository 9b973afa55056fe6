# round-3 batch: new GPU tests (bucketed all-reduce, deferred trunk weight gradients, PSNR),
# parity / bf16 / graph / variants on the TN changes, A/B of the deferral at 512 and 4096 rays,
# C5 trunk2=3, 2-rank shared-device bench, full psnr_long
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_flatgrad.py tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_psnr.py > gpurun_out/r3c_test.log 2>&1
for gb in 512 4096; do
for o in "" "--no-defer-wgrad" "" "--no-defer-wgrad"; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch $gb --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
echo "c4@$gb [$o] $r" >> gpurun_out/r3c_defer.log
done; done
CONFIG=c5 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=3" "trunk2=0" "trunk2=3" > gpurun_out/r3c_c5_trunk2.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-device --steps 10 --warmup 3 --no-secondary > gpurun_out/r3c_share2.json 2> gpurun_out/r3c_share2.err
timeout -k 10 600 python -u -c "
import json, bench
r = bench.psnr_long()
print(json.dumps(r))
" > gpurun_out/r3c_psnr_long.json 2> gpurun_out/r3c_psnr_long.err
