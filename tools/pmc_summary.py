"""Aggregate rocprofv3 --pmc counter CSVs per kernel (profiling infrastructure).

    python tools/pmc_summary.py gpurun_out/pmc1/p_counter_collection.csv [N]
    python tools/pmc_summary.py --traffic profiles/r01_traffic.json FETCH.csv WRITE.csv

--traffic writes, per kernel (named as bench.py / selunet_gemm_kernel_name name them), the HBM
bytes per launch: FETCH_SIZE x 2 (on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (exact for 16-B stores), both
in KiB units as rocprofv3 reports them.
"""
import csv
import json
import re
import sys
from collections import defaultdict

# rocprofv3 kernel-name pattern -> selunet kernel name (as bench.py names them). rocprofv3 prints
# fp32 instantiations demangled ("conv3x3_halo_persist_kernel<float, 128>") and bf16 ones mangled
# ("conv3x3_halo_persist_kernelIDF16bLi128E"): every entry matches both spellings.
_MANGLE = {"bf16": ("DF16b", "__bf16"), "f32": ("f", "float"), "true": ("Lb1E", "true")}


def _pat(base, *targs):
    m = "".join(_MANGLE[a][0] if a in _MANGLE else f"Li{a}E" for a in targs)
    d = ", ".join(_MANGLE[a][1] if a in _MANGLE else str(a) for a in targs)
    return rf"{base}I{m}|{re.escape(base + '<' + d)}[,>]" if targs else base


NAME_MAP = [
    (r"gemm_gather_kernelIfLi(128|64)ELb0ELb1E|gemm_gather_kernel<float, (128|64), false, true", "gemm_gather_x2<f32>"),
    (r"convt_x2_kernel", "gemm_gather_x2<f32>"),  # (the resident-weight ConvTranspose2d forward, same entry point)
    (r"convt_ring_x2_kernel", "gemm_gather_x2<f32>"),  # (the LDS-DMA ring ConvTranspose2d kernel, same entry point)
    (r"gemm_wgrad_x2_kernel", "gemm_wgrad_x2<f32>"),
    (_pat("conv3x3_halo_persist_kernel", "f32", 128, "true"), "conv3x3_x2<f32,128>"),
    (_pat("conv3x3_halo_persist_kernel", "f32", 64, "true"), "conv3x3_x2<f32,64>"),
    (r"conv3x3_x2d_kernel", "conv3x3_x2d<f32,64>"),
    (r"conv3x3_x2p_kernel", "conv3x3_x2p<f32,128>"),
    (r"convt_bf16_kernel(<\d+, \d+, false>|ILi\d+ELi\d+ELb0E)", "convt<bf16>"),
    (r"convt_bf16_kernel(<\d+, \d+, true>|ILi\d+ELi\d+ELb1E)", "convt_dgrad<bf16>"),
    (_pat("conv3x3_wgrad_x2_kernel", 128), "conv3x3_wgrad_x2<128>"),
    (_pat("conv3x3_wgrad_x2_kernel", 64), "conv3x3_wgrad_x2<64>"),
]
for _t in ("bf16", "f32"):
    NAME_MAP += [
        (_pat("conv3x3_halo_persist_kernel", _t, 128), f"conv3x3_halo_persist<{_t},128>"),
        (_pat("conv3x3_halo_persist_kernel", _t, 64), f"conv3x3_halo_persist<{_t},64>"),
        (_pat("conv3x3_halo_kernel", _t, 64, "true"), f"conv3x3_halo1<{_t},64>"),
        (_pat("conv3x3_halo_kernel", _t, 128), f"conv3x3_halo<{_t},128>"),
        (_pat("conv3x3_halo_kernel", _t, 64), f"conv3x3_halo<{_t},64>"),
        (_pat("gemm_gather_kernel", _t), f"gemm_gather<{_t}>"),
        (_pat("bn_bwd_apply_kernel", _t), f"bn_bwd_apply<{_t}>"),
        (_pat("bn_bwd_apply_pool_kernel", _t), f"bn_bwd_apply<{_t}>"),  # (dA formed on the fly: same entry in bench.py)
        (_pat("bn_bwd_apply_heads_kernel", _t), f"bn_bwd_apply<{_t}>"),
        (_pat("bn_bwd_apply_heads_planes_kernel", _t), f"bn_bwd_apply<{_t}>"),
        (_pat("maxpool_fwd_kernel", _t), f"maxpool2_fwd<{_t}>"),
        (_pat("maxpool_bwd_kernel", _t), f"maxpool2_bwd<{_t}>"),
        (_pat("heads_fwd_kernel", _t), f"heads_fwd<{_t}>"),
        (_pat("heads_bwd_kernel", _t), f"heads_bwd<{_t}>"),
        (_pat("first_conv_fwd_kernel", _t), f"first_conv_fwd<{_t}>"),
        (_pat("first_conv_wgrad_kernel", _t), f"first_conv_wgrad<{_t}>"),
    ]
NAME_MAP += [
    (_pat("conv3x3_wino_persist_kernel", 128), "conv3x3_wino<f32,128>"),
    (_pat("conv3x3_wino_persist_kernel", 64), "conv3x3_wino<f32,64>"),
    (_pat("conv3x3_wgrad_wino_f32_kernel", 16), "conv3x3_wgrad_wino_f32<64>"),
    (_pat("conv3x3_wgrad_wino_f32_kernel", 8), "conv3x3_wgrad_wino_f32<64>"),
    (_pat("conv3x3_wgrad_halo_f32_kernel", 128), "conv3x3_wgrad_halo_f32<128>"),
    (_pat("conv3x3_wgrad_halo_f32_kernel", 64), "conv3x3_wgrad_halo_f32<64>"),
    (_pat("conv3x3_wgrad_halo_kernel", 128), "conv3x3_wgrad_halo<128>"),
    (_pat("conv3x3_wgrad_halo_kernel", 64), "conv3x3_wgrad_halo<64>"),
    (r"gemm_wgrad_bf16_kernel", "gemm_wgrad_bf16"),
    (r"gemm_wgrad_kernel", "gemm_wgrad<f32>"),
]


def short(name):
    for pat, s in NAME_MAP:
        if re.search(pat, name):
            return s
    return name


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


def report(paths, top=12):
    agg, calls, dur = load(paths[0])
    for p in paths[1:]:  # counter passes of the same program, kernels matched by name
        a2, _, _ = load(p)
        for k, v in a2.items():
            for ctr, x in v.items():
                agg[k].setdefault(ctr, x)
    keys = sorted(agg, key=lambda k: -sum(dur[k].values()))
    for k in keys[:top]:
        c = agg[k]
        n = len(calls[k])
        t = sum(dur[k].values())
        line = f"{t / 1e6:8.2f} ms {n:4d} calls {short(k)[:40]:40s}"
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
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


def traffic(out, fetch_csv, write_csv):
    fa, fc, fd = load(fetch_csv)
    wa, wc, wd = load(write_csv)
    res = {}
    per = defaultdict(lambda: {"fetch": 0.0, "write": 0.0, "calls_f": 0, "calls_w": 0, "ns": 0})
    for k in fa:
        s = short(k)
        per[s]["fetch"] += fa[k]["FETCH_SIZE"] * 1024 * 2
        per[s]["calls_f"] += len(fc[k])
        per[s]["ns"] += sum(fd[k].values())
    for k in wa:
        s = short(k)
        per[s]["write"] += wa[k]["WRITE_SIZE"] * 1024
        per[s]["calls_w"] += len(wc[k])
    for s, v in per.items():
        if v["calls_f"] == 0 or v["calls_w"] == 0:
            continue
        f = v["fetch"] / v["calls_f"]
        w = v["write"] / v["calls_w"]
        res[s] = {"hbm_bytes_per_launch": f + w, "fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
                  "launches": v["calls_f"], "avg_launch_us": v["ns"] / v["calls_f"] / 1e3}
    doc = {"method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; "
                     "bytes = FETCH_SIZE*1024*2 (gfx950 half-count correction) + WRITE_SIZE*1024, per launch",
           "sources": [fetch_csv, write_csv], "kernels": res}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(f"wrote {out}: {len(res)} kernels")


if __name__ == "__main__":
    if sys.argv[1] == "--traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        report([a for a in sys.argv[1:] if a.endswith(".csv")],
               int(sys.argv[-1]) if not sys.argv[-1].endswith(".csv") else 12)
