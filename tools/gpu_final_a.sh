# end of round 3: the GPU suite, then the bench lines of the final tree (default C4 with the CPU
# baseline and the long PSNR study, C4 at 512 rays, C3, C5) and a trunk2=1 training A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/final/gputest.log | head -20; tail -20 gpurun_out/final/gputest.log; exit 1; }
tail -1 gpurun_out/final/gputest.log
timeout -k 10 560 python -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { echo "BENCH FAILED"; tail -20 gpurun_out/final/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench_default.json')); print('C4', d['ms_per_step'], d['value'], d['roofline']['kernel'][:30], d['roofline']['frac'], 'mlp', d['mlp_mfma_utilisation']['frac'])"
timeout -k 10 200 python bench.py --config c4 --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/final/bench_c4_512.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-secondary > gpurun_out/final/bench_c3.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-secondary > gpurun_out/final/bench_c5.json 2>/dev/null || exit 1
for f in c4_512 c3 c5; do python -c "import json; d=json.load(open('gpurun_out/final/bench_$f.json')); print('$f', d['ms_per_step'], d['value'], d['roofline']['kernel'][:30], d['roofline']['frac'], (d.get('mlp_mfma_utilisation') or {}).get('frac'))"; done
bash tools/gpu_ab_opt.sh "trunk2=3" "trunk2=1 trunk2_tile=64"
