"""Kernel statistics and per-step idle gaps from a rocprofv3 rocpd database (profiling tool).

    python tools/rocpd_stats.py gpurun_out/p16/run_results.db [--csv out.csv] [--steps 10] [--gaps 15]

--csv writes the same columns as `rocprofv3 --stats` (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev). The step report takes the last `--steps` training steps (a step
ends at an `adam_kernel` dispatch) and splits each step's wall span into kernel time and the idle
gaps between consecutive dispatches, listing the largest gaps by the kernel that follows them.
"""
import argparse
import csv
import sqlite3
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gaps", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    per = defaultdict(list)
    for name, s, e in rows:
        per[name].append(e - s)
    tot = sum(sum(v) for v in per.values())
    if a.csv:
        with open(a.csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
            for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v),
                            statistics.pstdev(v) if len(v) > 1 else 0.0])
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    if len(ends) < a.steps + 1:
        print(f"{len(ends)} steps in the trace")
        return
    lo, hi = ends[-a.steps - 1], ends[-1]
    span = rows[hi][2] - rows[lo][2]
    busy = sum(rows[i][2] - rows[i][1] for i in range(lo + 1, hi + 1))
    gaps = defaultdict(list)
    prev_end = rows[lo][2]
    for i in range(lo + 1, hi + 1):
        g = rows[i][1] - prev_end
        gaps[rows[i][0]].append(max(g, 0))
        prev_end = max(prev_end, rows[i][2])
    n = a.steps
    print(f"{n} steps: {span / n / 1e6:.3f} ms/step wall, kernels {busy / n / 1e6:.3f} ms, "
          f"gaps {(span - busy) / n / 1e6:.3f} ms, {(hi - lo) / n:.0f} dispatches/step")
    print("largest gap totals per step (before the named kernel):")
    for name, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:a.gaps]:
        print(f"  {sum(v) / n / 1e3:8.1f} us  {len(v) // n:4d}x  {name[:100]}")
    print("kernel time per step:")
    kt = defaultdict(int)
    for i in range(lo + 1, hi + 1):
        kt[rows[i][0]] += rows[i][2] - rows[i][1]
    for name, v in sorted(kt.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {v / n / 1e3:8.1f} us  {name[:100]}")


if __name__ == "__main__":
    main()
