# SQ stall breakdown of the weight-gradient lab kernels (tools/tn_lab mode 1..5), one PMC pass per
# counter group: bash tools/pmc_tn_lab.sh
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_tn
mkdir -p $OUT
for m in 1 2 5; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $OUT/m$m -o p -- ./tools/tn_lab 1048576 5 $m > $OUT/m$m.log 2>&1 || { tail -5 $OUT/m$m.log; exit 1; }
  python3 - $OUT/m$m <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tn_bf16" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
w = acc["SQ_WAVE_CYCLES"]
print(sys.argv[1].split("/")[-1], {k: round(v / w, 3) if k != "SQ_WAVE_CYCLES" else v for k, v in sorted(acc.items())})
PY
done
