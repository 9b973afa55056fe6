"""Per-launch HBM traffic of every kernel class from tools/pmc_bench.sh output, with the gfx950
correction of MI355X_MICROARCH.md §HBM: bytes = 2 × FETCH_SIZE + WRITE_SIZE (both in KiB).
Writes <dst>/traffic_<cfg>_rays<N>.json — keyed by the workload AND its rays per rank, so that
bench.py's roofline.traffic is only ever the profile of the same batch size.
    python tools/traffic_summary.py gpurun_out/pmc_bench profiles/r03 c4:4096 c4:512 c5:32768"""
import collections
import csv
import glob
import json
import os
import re
import sys

# rocprof kernel name → the library's profiling class (one class per kernel function)
CLASSES = [(r"k_gemm_nt_bf16d<true", "gemm_nt_bf16d_dmul"), (r"k_gemm_nt_bf16d<", "gemm_nt_bf16d"),
           (r"k_gemm_nt_bf16w", "gemm_nt_bf16w"), (r"k_gemm_nt_bf16<", "gemm_nt_bf16"),
           (r"k_gemm_tn_bf16_k64", "gemm_tn_bf16k"), (r"k_gemm_tn_bf16d", "gemm_tn_bf16d"), (r"k_gemm_tn_bf16w", "gemm_tn_bf16w"), (r"k_gemm_tn_bf16\b", "gemm_tn_bf16"),
           (r"k_gemm_nt_w<|k_gemm_nt<", "gemm_nt_f32"), (r"k_gemm_tn<", "gemm_tn_f32"),
           (r"k_trunk_bf16<128, 2048", "trunk_bf16_train"), (r"k_trunk_bf16<128, (4096|36864)", "trunk_heads_bf16"), (r"k_trunk_bf16<128", "trunk_bf16"), (r"k_trunk_bf16<64", "trunk_bf16_train"),
           (r"k_trunk2_bf16<\d+, (true|false), true", "trunk_bf16_train"),
           (r"k_trunk2_bf16<\d+, (true|false), false, true", "trunk_heads_bf16"), (r"k_trunk2_bf16<", "trunk_bf16"),
           (r"k_trunk_bwd_bf16", "trunk_bwd_bf16"), (r"k_heads_train_bf16", "heads_train"), (r"k_heads_bf16", "heads_fused"),
           (r"k_heads_fwd", "heads_fwd"), (r"k_heads_bwd", "heads_bwd"), (r"k_tn_skinny", "tn_skinny"),
           (r"k_reduce_slabs", "reduce_slabs"), (r"k_encode", "encode"), (r"k_composite_fwd", "composite_fwd"),
           (r"k_composite_bwd", "composite_bwd"), (r"k_ray_rowsum", "ray_rowsum"),
           (r"k_merge_rows", "merge_samples"), (r"k_heads_dx_bf16", "heads_dx")]


def class_of(name):
    for pat, cls in CLASSES:
        if re.search(pat, name):
            return cls
    return None


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_bench"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r03"
    RUNS = sys.argv[3:] or ["c4:4096", "c5:32768"]
    for run in RUNS:
        cfg, rays = run.split(":")
        tag = f"{cfg}_rays{rays}"
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            for f in glob.glob(os.path.join(src, f"{tag}_{ctr}", "**", "*counter_collection.csv"), recursive=True):
                per = collections.defaultdict(float)
                names = {}
                for r in csv.DictReader(open(f)):
                    d = int(r["Dispatch_Id"])
                    per[d] += float(r["Counter_Value"])
                    names[d] = r["Kernel_Name"]
                for d, v in per.items():
                    cls = class_of(names[d])
                    if cls:
                        acc[cls][ctr].append(v)
        out = {}
        for cls, c in acc.items():
            if not c.get("FETCH_SIZE") or not c.get("WRITE_SIZE"):
                continue
            fetch = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
            write = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
            out[cls] = {"launches": len(c["FETCH_SIZE"]), "hbm_read_bytes_per_launch": fetch,
                        "hbm_write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
                        "rays_per_rank": int(rays),
                        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over `bench.py --config "
                                  f"{cfg} --global-batch {rays} --eager --steps 2 --warmup 1`; bytes = 2*FETCH_SIZE + "
                                  "WRITE_SIZE (KiB, gfx950 correction, MI355X_MICROARCH.md HBM)"}
        if out:
            os.makedirs(dst, exist_ok=True)
            json.dump(out, open(os.path.join(dst, f"traffic_{tag}.json"), "w"), indent=1)
            print(tag, {k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in out.items()}, "MB/launch")


if __name__ == "__main__":
    main()
