# round-3 check: new GPU tests (Philox ranks, flat grads, losses, bf16 per-key bounds, PSNR), then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a_gputest.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" gpurun_out/r3a_gputest.log | head -30; tail -30 gpurun_out/r3a_gputest.log; exit 1; }
tail -3 gpurun_out/r3a_gputest.log
timeout -k 10 900 python bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/r3a_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3a_bench.json')); print('C4', d['ms_per_step'], d['value'], d['roofline']['kernel'][:40], d['roofline']['frac'], d['mlp_mfma_utilisation']['frac']); print(d['cpu_baseline']); print({k: v for k, v in d['psnr_long'].items() if k != 'loss_curve'})"
