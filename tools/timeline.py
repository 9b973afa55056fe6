"""Timeline of the bench's last training steps from a rocprofv3 --kernel-trace CSV (a file or a
directory holding one): per step the span (Adam end to Adam end), the kernels' summed time, the
time at least one kernel runs (the union over queues) and the idle gaps between them, then the
last step's kernel sequence with start offsets and queues and its per-kernel summary — where a
step's time goes that no per-kernel average shows.

    python tools/timeline.py gpurun_out/<dir> [steps=8] [gap_us=3]
"""
import collections
import csv
import glob
import sys


def short(name):
    n = name.replace("void ", "").split("(")[0]
    return n.replace("spn::", "")[:58]


def main():
    path = sys.argv[1]
    if not path.endswith(".csv"):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[0]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    gap_min = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Queue_Id", "?"), int(r.get("Grid_Size_X", 0))))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "k_adam" in r[2]]
    if len(ends) < 2:
        sys.exit(f"only {len(ends)} k_adam launches in {path}")
    ends = ends[-(min(nsteps, len(ends) - 1) + 1):]
    tot_span = tot_busy = tot_sum = 0.0
    worst = []
    for a, b in zip(ends, ends[1:]):
        t0 = rows[a][1]
        ks = [r for r in rows[a + 1:b + 1] if r[1] > t0]
        span = (rows[b][1] - t0) / 1e3
        ksum = sum(r[1] - r[0] for r in ks) / 1e3
        busy, cur_end, gaps = 0.0, t0, []
        prev = rows[a]
        for r in ks:
            if r[0] > cur_end:
                g = (r[0] - cur_end) / 1e3
                if g >= gap_min:
                    gaps.append((g, short(prev[2]), short(r[2])))
            s = max(r[0], cur_end)
            if r[1] > s:
                busy += (r[1] - s) / 1e3
            if r[1] > cur_end:
                cur_end, prev = r[1], r
        idle = span - busy
        tot_span += span
        tot_busy += busy
        tot_sum += ksum
        print(f"step: span {span:8.1f} us  kernels {len(ks):3d}  sum {ksum:8.1f}  busy {busy:8.1f}  idle {idle:7.1f}"
              f"  gaps>={gap_min:g}us {len(gaps)} ({sum(g[0] for g in gaps):.1f} us)")
        worst = gaps
    n = len(ends) - 1
    print(f"mean: span {tot_span / n:.1f} us, kernel sum {tot_sum / n:.1f}, busy {tot_busy / n:.1f}, idle {(tot_span - tot_busy) / n:.1f}")
    print("\nlargest gaps of the last step (us, kernel before -> kernel after):")
    for g in sorted(worst, reverse=True)[:25]:
        print(f"  {g[0]:7.1f}  {g[1]} -> {g[2]}")
    a, b = ends[-2], ends[-1]
    t0 = rows[a][1]
    print("\nlast step's kernels (start offset us, duration us, queue, grid, name):")
    for r in rows[a + 1:b + 1]:
        print(f"  {(r[0] - t0) / 1e3:8.1f} {(r[1] - r[0]) / 1e3:8.1f}  q{r[3]:>3s} {r[4]:8d}  {short(r[2])}")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[a + 1:b + 1]:
        agg[short(r[2])][0] += 1
        agg[short(r[2])][1] += (r[1] - r[0]) / 1e3
    tot = sum(v[1] for v in agg.values())
    print("\nlast step per kernel (us, launches, share):")
    for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {d:9.1f} {n:4d}x {100 * d / tot:5.1f}%  {name}")


if __name__ == "__main__":
    main()
