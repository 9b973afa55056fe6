"""Summarise tools/pmc_gemm*.sh output: one line of derived counters per (kernel, grid).
    python tools/pmc_summary.py gpurun_out/pmc16
PMC_MATCH (a regex, default "gemm|trunk") and PMC_MIN_GRID (default 100000) pick the kernels."""
import collections
import re
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc16"
data, meta = collections.defaultdict(dict), {}
for f in sorted(glob.glob(os.path.join(root, "p*", "p_counter_collection.csv"))):
    # each pass is its own run of the same command (same dispatch sequence): a counter's value sums
    # its per-instance rows within one pass; counters another pass collected already are not re-added
    have = {d: set(c) for d, c in data.items()}
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        if r["Counter_Name"] in have.get(d, ()):
            continue
        data[d][r["Counter_Name"]] = data[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        meta.setdefault(d, (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
seen = set()
for d in sorted(data):
    name, grid, dur = meta[d]
    short = name.split("(")[0].replace("void spn::", "").replace("spn::", "")
    if not re.search(os.environ.get("PMC_MATCH", "gemm|trunk"), short) or grid < int(os.environ.get("PMC_MIN_GRID", 100000)) \
            or (short, grid) in seen:
        continue
    seen.add((short, grid))
    c = data[d]
    W = c.get("SQ_WAVES", 1)
    wc = c.get("SQ_WAVE_CYCLES", 1)
    gui = c.get("GRBM_GUI_ACTIVE", 1) / 8  # summed over the 8 XCDs
    print(f"{short:24s} grid={grid:8d} dur={dur / 1e3:7.1f}us clk={gui / dur:.2f}GHz cyc/wave={4 * wc / W:.0f} valu/wave={c.get('SQ_INSTS_VALU', 0) / W:.0f} "
          f"lds/wave={c.get('SQ_INSTS_LDS', 0) / W:.0f} mfma/wave={c.get('SQ_INSTS_MFMA', 0) / W:.0f}")
    print(f"    waitAny {c.get('SQ_WAIT_ANY', 0) / wc:.2f} waitInst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"(lds {c.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}) active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
          f"mfma-busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui * 1024):.2f} "
          f"ldsconf {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c.get('SQ_LDS_IDX_ACTIVE', 1)):.3f} "
          f"FETCHx2 {2 * c.get('FETCH_SIZE', 0) * 1024 / 1e6:.0f}MB WRITE {c.get('WRITE_SIZE', 0) * 1024 / 1e6:.0f}MB")
