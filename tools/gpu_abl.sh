# GPU-box: trunk k-walk rotation A/B
set -o pipefail
mkdir -p gpurun_out
for opt in "--option trunk_rot=0" "--option trunk_rot=1" "--option trunk_rot=0 --option trunk_dbg=1" "--option trunk_rot=1 --option trunk_dbg=1"; do
  echo "== $opt"
  timeout -k 10 200 python tools/trunk_bench.py $opt > gpurun_out/tb.txt 2>&1 || { cat gpurun_out/tb.txt; exit 1; }
  grep -E "^(save|nosave)" gpurun_out/tb.txt | sed -e "s/'gemm_nt_bf16.*//"
done
