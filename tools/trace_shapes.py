"""Per-launch-shape durations of chosen kernels from a rocprofv3 --kernel-trace CSV: the
default bench command also runs C2, the PSNR parity and its small renders, so rocprof's
per-kernel averages mix shapes; this separates them by grid size (the bench workload's launches
are the large grids).

    python tools/trace_shapes.py gpurun_out/prof_default/p_kernel_trace.csv k_trunk_bf16 k_trunk_bwd_bf16
"""
import collections
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        key = next((k for k in keys if k + "<" in name or k + "(" in name), None)
        if key is None:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g[(name.split("(spn")[0].replace("void ", ""), int(r["Grid_Size_X"]))].append(d)
    print(f"{'kernel':40s} {'grid':>8s} {'launches':>8s} {'min_us':>9s} {'median_us':>9s} {'mean_us':>9s} {'max_us':>9s}")
    for (name, grid), v in sorted(g.items()):
        v.sort()
        print(f"{name[:40]:40s} {grid:8d} {len(v):8d} {v[0]:9.1f} {v[len(v) // 2]:9.1f} {sum(v) / len(v):9.1f} {v[-1]:9.1f}")


if __name__ == "__main__":
    main()
