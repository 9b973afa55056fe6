"""Per-launch HBM traffic of the GEMM classes from tools/pmc_bench.sh output, with the gfx950
correction of MI355X_MICROARCH.md §HBM: bytes = 2 × FETCH_SIZE + WRITE_SIZE (both in KiB).
Writes <dst>/traffic_<cfg>.json for bench.py's roofline.traffic.
    python tools/traffic_summary.py gpurun_out/pmc_bench profiles/r02 c4 c5"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_bench"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r02"
CFGS = sys.argv[3:] or ["c4", "c5"]
CLASSES = {"k_gemm_nt<": "gemm_nt_f32", "k_gemm_nt_w<": "gemm_nt_f32", "k_gemm_tn<": "gemm_tn_f32",
           "k_gemm_nt_bf16": "gemm_nt_bf16", "k_gemm_tn_bf16": "gemm_tn_bf16", "k_trunk_bf16<128": "trunk_bf16", "k_trunk_bf16<64": "trunk_bf16_train",
           "k_trunk_bwd_bf16": "trunk_bwd_bf16",
           "k_heads_bf16": "heads_fused", "k_composite_fwd": "composite_fwd"}
for cfg in CFGS:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(os.path.join(src, f"{cfg}_{ctr}", "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                d = int(r["Dispatch_Id"])
                per[d] += float(r["Counter_Value"])
                names[d] = r["Kernel_Name"]
            for d, v in per.items():
                for key, cls in CLASSES.items():
                    if key in names[d] and not ("bf16" in names[d] and cls.endswith("_f32")):
                        acc[cls][ctr].append(v)
    out = {}
    for cls, c in acc.items():
        if not c.get("FETCH_SIZE") or not c.get("WRITE_SIZE"):
            continue
        fetch = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        write = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        out[cls] = {"launches": len(c["FETCH_SIZE"]), "hbm_read_bytes_per_launch": fetch,
                    "hbm_write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
                    "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --config "
                              f"{cfg} --eager --steps 2 --warmup 1`; bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB, gfx950 "
                              "correction, MI355X_MICROARCH.md HBM)"}
    if out:
        os.makedirs(dst, exist_ok=True)
        json.dump(out, open(os.path.join(dst, f"traffic_{cfg}.json"), "w"), indent=1)
        print(cfg, {k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in out.items()}, "MB/launch")
