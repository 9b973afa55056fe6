# round 3 (session 2): tile row sums fused into the dX chain, balanced TN bias — parity tests, then A/B pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_bf16.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread -k "fused_backward or tile_rowsum or bias_split or tilings or bf16 or dp" > gpurun_out/r3i_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3i_tests.log | head -20; tail -5 gpurun_out/r3i_tests.log; exit 1; }
tail -1 gpurun_out/r3i_tests.log
bash tools/gpu_ab_opt.sh "tile_rowsum=0 tn_bf16_bias_split=0" "tile_rowsum=1 tn_bf16_bias_split=0" "tile_rowsum=1 tn_bf16_bias_split=1" "tile_rowsum=0 tn_bf16_bias_split=0" "tile_rowsum=1 tn_bf16_bias_split=1"
GB=512 bash tools/ab512.sh "tile_rowsum=0 tn_bf16_bias_split=0" "tile_rowsum=1 tn_bf16_bias_split=1" "tile_rowsum=0 tn_bf16_bias_split=0" "tile_rowsum=1 tn_bf16_bias_split=1"
export TMPDIR=/tmp
for bsv in 0 1; do
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r3i_pmc_bs$bsv -o p -- python3 bench.py --config c4 --global-batch 4096 --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --option tn_bf16_bias_split=$bsv > gpurun_out/r3i_pmc_bs$bsv.log 2>&1 || { echo "PMC FAILED"; tail -5 gpurun_out/r3i_pmc_bs$bsv.log; exit 1; }
done
echo PMC done
