"""Per-launch mean of one PMC counter by kernel class (tools/pmc_dx.sh): for FETCH_SIZE the HBM read
bytes with the gfx950 correction (2 × KiB), in GB.
    python tools/pmc_dx_summary.py gpurun_out/pmc_dx/run1"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic_summary import class_of  # noqa: E402  (the classes only; its main loop needs argv)

per = collections.defaultdict(float)
names = {}
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        per[d, r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
acc = collections.defaultdict(list)
for (d, ctr), v in per.items():
    c = class_of(names[d])
    if c:
        acc[ctr, c].append(v)
for ctr in sorted({k[0] for k in acc}):
    scale = 2 * 1024 / 1e9 if ctr == "FETCH_SIZE" else (1024 / 1e9 if ctr == "WRITE_SIZE" else 1.0)
    out = {c: round(scale * sum(v) / len(v), 3) for (k, c), v in sorted(acc.items()) if k == ctr and sum(v) > 0}
    print(ctr, out)
