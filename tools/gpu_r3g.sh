# end-of-round bench lines: the default command (C4 + C2 + CPU baseline + PSNR parity + long PSNR),
# C4 at 512 rays per rank, C3, C5
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err
timeout -k 10 300 python bench.py --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/final/bench_c4_512.json 2> gpurun_out/final/bench_c4_512.err
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/final/bench_c3.json 2> gpurun_out/final/bench_c3.err
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/final/bench_c5.json 2> gpurun_out/final/bench_c5.err
