"""Emulate the overlapped gradient all-reduce on one GPU.

The 8-GPU run issues one RCCL all-reduce per gradient bucket while the backward continues; RCCL's
kernel holds some CUs for the length of the collective. This tool runs the bench step
(SelectiveUNet_B fp32, s_lamb 2, synthetic HBM-resident batch) at a per-GPU batch B and, at every
point GradBucketer fires, launches `selunet_cu_hold` (n_wg workgroups reduce-copying the bucket for
`us` microseconds) on a side stream (parallel.OverlapEmulation). It prints, per setting, the step
time, the inflation over the plain step, the side-stream time of the stand-in kernels (start of
dispatch to end, so waiting for CUs counts) and their own CU-time (n_wg x us).

    python tools/overlap_emulation.py --batch 16 --cases 0:0,16:100,32:100,16:300,32:300
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import parallel  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2, help="alternating repetitions of the whole case list")
    ap.add_argument("--cases", default="0:0,16:100,32:100,16:300,32:300",
                    help="comma list of n_wg:us (0:0 = no stand-in kernel)")
    ap.add_argument("--bucket-mb", default="4", help="comma list of bucket sizes (MB of fp32 gradients)")
    ap.add_argument("--option", action="append", default=[], help="KEY=VALUE library option (selunet_set_option)")
    ap.add_argument("--halo-wgs", type=int, default=0, help="selunet_set_halo_workgroups (0: default 256)")
    ap.add_argument("--model", default="", help="alpha_us:beta_GBs — each stand-in holds its CUs for alpha + "
                    "bucket bytes / beta (a bandwidth model of the all-reduce) instead of the case's fixed us")
    ap.add_argument("--priority", type=int, default=0, help="run the step on a stream of this priority "
                    "(-1: high; the stand-in's side stream stays at the default)")
    ap.add_argument("--side-priority", type=int, default=0, help="the stand-in's side stream priority (-1: high, "
                    "as ProcessGroupNCCL.Options(is_high_priority_stream=True) gives RCCL's streams)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K.load()
    for kv in a.option:
        k, v = kv.split("=")
        K.set_option(k, int(v))
    if a.halo_wgs:
        K.load().selunet_set_halo_workgroups(a.halo_wgs)
    x, lab = make_batch(a.batch, 256, seed=1)
    xt, lt = torch.tensor(x, device=dev), torch.tensor(lab, device=dev)
    net = S.UNet_B("RGB", selective=True)
    p = L.seeded_params(0, "RGB", True, bn_affine_random=False)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(dev).train()
    opt = S.Adam(net.parameters(), lr=1e-3)
    loss_a = S.BCEWithLogitsLoss()

    cstream = torch.cuda.Stream(device=dev, priority=a.priority) if a.priority else None
    model = tuple(float(v) for v in a.model.split(":")) if a.model else None

    def step():
        if cstream is not None:
            with torch.cuda.stream(cstream):
                return step_()
        return step_()

    def step_():
        out, sel, aux = net(xt)
        loss = loss_a(aux, lt) + S.calc_selective_risk_image_b(out, sel, target=lt, lamb=2)[0]
        opt.zero_grad()
        loss.backward()
        opt.step()

    cases = []
    for mb in a.bucket_mb.split(","):
        for c in a.cases.split(","):
            n_wg, us = c.split(":")
            cases.append((int(float(mb) * (1 << 18)), int(n_wg), float(us)))
    for _ in range(a.warmup):
        step()
    res = {c: [] for c in cases}
    side = {c: [] for c in cases}
    nb, held = {}, {}
    for rep in range(a.reps):
        for c in cases:
            belems, n_wg, us = c
            parallel.set_bucket_elems(belems)
            emu = (parallel.OverlapEmulation(n_wg, us, timing=True, model=model, priority=a.side_priority)
                   if n_wg > 0 else None)
            parallel.set_overlap_emulation(emu)
            step()  # a fresh plan key is not needed: the markers are host hooks between graph segments
            torch.cuda.synchronize()
            if emu is not None:
                emu.events.clear()
                emu.held_us = 0.0
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            res[c].append(dt)
            if emu is not None:
                side[c].append(sum(e0.elapsed_time(e1) for _, e0, e1 in emu.events) / a.steps)
                nb[c] = len(emu.events) // a.steps
                held[c] = emu.held_us / a.steps
            parallel.set_overlap_emulation(None)
    parallel.set_bucket_elems(1 << 20)
    rows = []
    base = {}
    for c in cases:
        belems, n_wg, us = c
        ms = 1e3 * min(res[c])
        if n_wg == 0:
            base[belems] = ms
    for c in cases:
        belems, n_wg, us = c
        ms = 1e3 * min(res[c])
        b0 = base.get(belems, min(base.values()) if base else ms)
        nbk = nb.get(c, 0)
        row = {"bucket_mb": belems / (1 << 18), "n_wg": n_wg, "us": us, "buckets": nbk,
               "ms_per_step": round(ms, 3), "all_ms": [round(1e3 * v, 3) for v in res[c]],
               "inflation_ms": round(ms - b0, 3),
               "standin_wall_ms": round(held.get(c, 0.0) / 1e3, 3),
               "standin_side_ms": round(min(side[c]), 3) if side[c] else 0.0,
               "standin_cu_share_ms": round(held.get(c, 0.0) / 1e3 * n_wg / 256, 3)}
        rows.append(row)
        print(f"{'model ' + a.model + ' ' if model else ''}prio {a.priority} side {a.side_priority} halo {a.halo_wgs or 256} "
              f"bucket {row['bucket_mb']:5.1f} MB  n_wg {n_wg:3d}  us {us:6.0f}  buckets {nbk:2d}  "
              f"{ms:8.3f} ms/step  inflation {row['inflation_ms']:7.3f} ms  stand-in wall {row['standin_wall_ms']:6.3f} ms "
              f"(side stream {row['standin_side_ms']:6.3f}, CU share {row['standin_cu_share_ms']:6.3f})", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": a.batch, "steps": a.steps, "options": a.option, "halo_wgs": a.halo_wgs, "model": a.model,
                       "priority": a.priority, "side_priority": a.side_priority, "rows": rows}, f,
                      indent=1)


if __name__ == "__main__":
    main()
