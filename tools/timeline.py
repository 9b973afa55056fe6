"""One training step's kernel sequence from a rocprofv3 --kernel-trace CSV (the launches between
the last two k_adam calls), with durations and a per-kernel summary.

    python tools/timeline.py gpurun_out/<dir>/<...>_kernel_trace.csv [--all]
"""
import collections
import csv
import glob
import sys


def main():
    path = sys.argv[1]
    if not path.endswith(".csv"):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    a, b = (ends[-2] + 1, ends[-1] + 1) if len(ends) >= 2 else (0, len(rows))
    step = rows[a:b]
    tot = 0.0
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        name = r["Kernel_Name"][:100]
        agg[name][0] += 1
        agg[name][1] += d
        if "--all" in sys.argv:
            print(f"{d:9.1f}  grid={r.get('Grid_Size', r.get('Grid_Size_X', '?')):>8}  {name}")
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"# {len(step)} kernels, busy {tot:.1f} us, span {span:.1f} us")
    for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{d:9.1f} us {n:4d}x  {100 * d / tot:5.1f}%  {name}")


if __name__ == "__main__":
    main()
