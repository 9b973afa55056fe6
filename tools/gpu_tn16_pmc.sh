# GPU-box: bf16 TN tilings on the microbenchmark — checks + timings, then PMC passes (one counter
# group per pass, kernel-trace only) over the same run.
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_tn16
mkdir -p $OUT
timeout -k 10 120 ./tools/gemm_bench_bf16 131072 20 tn > $OUT/timing.txt 2>&1 || { cat $OUT/timing.txt; exit 1; }
cat $OUT/timing.txt
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- ./tools/gemm_bench_bf16 131072 3 tn > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc" >> $OUT/summary.txt
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob, collections
out = "gpurun_out/pmc_tn16"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_tn" not in k: continue
        agg[k.split("(")[0] + " grid=" + r.get("Grid_Size", "?")][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out + "/pmc_summary.txt", "w") as fh:
    for k, d in agg.items():
        line = k + " " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items()))
        print(line); fh.write(line + "\n")
PY
