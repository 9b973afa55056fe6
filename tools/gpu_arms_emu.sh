set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16.py > gpurun_out/red_test.log 2>&1
bash tools/ab512.sh "" "tn_bf16_variant=1" "tn_bf16_variant=1 tn_bf16_min_points=2048" "tn_bf16_variant=1 tn_bf16_min_points=4096" "tn_bf16_variant=2" > gpurun_out/ab512_tn.log 2>&1
bash tools/gpu_timeline.sh tl3 512 4096
timeout -k 10 900 python -u tools/psnr_arms.py --steps 1000 --batch 2048 --n-eval 4096 --seeds 3,4,5 --kinds fp32,bf16,emu > gpurun_out/arms_seeds.log 2>&1
