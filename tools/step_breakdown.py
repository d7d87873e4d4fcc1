"""Per-step kernel breakdown of a rocprofv3 --kernel-trace CSV (profiling tool): the last N steps,
delimited by heads_fwd launches (one per training step), per kernel name and in total.

    python tools/step_breakdown.py gpurun_out/prof/p_kernel_trace.csv [N] [out.txt]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    heads = [i for i, r in enumerate(rows) if "heads_fwd" in r["Kernel_Name"]]
    a, b = heads[-nsteps - 1], heads[-1]
    win = rows[a:b]
    tot = collections.defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:80]
        tot[name][0] += d
        tot[name][1] += 1
        busy += d
    wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6
    lines = [f"steps {nsteps}: wall {wall / nsteps:.3f} ms/step, kernel busy {busy / nsteps:.3f} ms/step, "
             f"{len(win) / nsteps:.0f} launches/step"]
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        lines.append(f"{v[0] / nsteps:8.3f} ms {v[1] // nsteps:4d}  {k}")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")


if __name__ == "__main__":
    main()
