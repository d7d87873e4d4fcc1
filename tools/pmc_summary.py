"""Aggregate rocprofv3 --pmc counter CSVs per kernel (test/profiling infrastructure)."""
import csv
import sys
from collections import defaultdict


def load(path):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    dur = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
        dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return agg, calls, dur


if __name__ == "__main__":
    agg, calls, dur = load(sys.argv[1])
    keys = sorted(agg, key=lambda k: -sum(dur[k].values()))
    for k in keys[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
        c = agg[k]
        n = len(calls[k])
        t = sum(dur[k].values())
        line = f"{t / 1e6:8.2f} ms {n:4d} calls {k[:60]:60s}"
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            line += (f" wait {c['SQ_WAIT_ANY'] / wc:5.2f} waitinst {c['SQ_WAIT_INST_ANY'] / wc:5.2f} "
                     f"active {c['SQ_ACTIVE_INST_ANY'] / wc:5.2f} ldsconf/wc {c['SQ_LDS_BANK_CONFLICT'] / wc:6.3f}")
            if "GRBM_GUI_ACTIVE" in c:
                # MFMA busy fraction of the 4 SIMDs x 256 CUs over the kernel's GPU-active cycles
                gpu = c["GRBM_GUI_ACTIVE"] / 8.0
                line += f" mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (gpu * 1024):5.3f} clk {gpu / (t / 1e9) / 1e9:4.2f}GHz"
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            if ctr in c:
                line += f" {ctr} {c[ctr] * 1024 / n / 1e6:9.1f} MB/call"
        print(line)
