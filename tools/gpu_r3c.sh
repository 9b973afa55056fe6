# round-3 batch 1: new GPU tests (bucketed all-reduce, deferred trunk weight gradients, NT epilogue
# variants, PSNR), parity / bf16 / graph / variants, A/B of the deferral and the NT epilogue
# variants at 512 and 4096 rays
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_flatgrad.py tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_psnr.py > gpurun_out/r3c_test.log 2>&1
for gb in 512 4096; do
for o in "" "--no-defer-wgrad" "--option nt_bf16_epi=0" "" "--no-defer-wgrad" "--option nt_bf16_epi=0"; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch $gb --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print(round(d['ms_per_step'],3), {c: round(v['ms_per_step'],3) for c, v in k.items() if v['ms_per_step'] > 0.1})")
echo "c4@$gb [$o] $r" >> gpurun_out/r3c_defer.log
done; done
timeout -k 10 300 python bench.py --gpus 2 --share-device --steps 10 --warmup 3 --no-secondary > gpurun_out/r3d_share2.json 2> gpurun_out/r3d_share2.err
