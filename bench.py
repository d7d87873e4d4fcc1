"""Benchmark: SelectiveUNet_B training images/sec, 256x256, global batch 128 (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]                       # N = 1
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N  # N > 1 (RCCL)

One step = the reference's training iteration (train.py:186-209) on synthetic, HBM-resident
data: forward of UNet_B(selective=True), BCEWithLogits aux loss + calc_selective_risk_image_b
(s_lamb=2), backward (with the RCCL gradient all-reduce when N > 1) and the Adam update. The
global batch of 128 is split into contiguous per-rank chunks (DataParallel semantics), so
`scaling` is "strong". Rank 0 prints one JSON line. The `roofline` object is for the dominant
kernel (the largest total time among the MFMA GEMM entry points, timed with HIP events on
the launch stream over the whole timed region); `cpu_baseline` times the CPU oracle
(oracle/unet_b_cpu.py, the reference's op sequence in torch eager on the host cores) on a
bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import parallel  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402

TRAIN_GFLOP_PER_IMG_256 = 220.38  # fwd 73.535 x 3 - first-layer dgrad
PEAK = {"bf16": (2500.0, "TFLOP/s"), "fp32": (157.3, "TFLOP/s")}  # MI355X dense MFMA (MICROARCH guide)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="global batch (split over ranks)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--lamb", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--layer-report", action="store_true", help="print per-entry-point timing to stderr")
    return ap.parse_args()


class KernelTimer:
    """Brackets the MFMA GEMM entry points with HIP events on the launch stream (torch's current
    stream, the one the kernels are launched on) and attributes each launch to the kernel it
    dispatches to (selunet_gemm_kernel_name), with its algorithmic FLOPs (2*M*N*K of the true,
    unpadded GEMM) and algorithmic HBM bytes (each operand tensor read once, output written once)."""

    ENTRY = ("selunet_gemm_gather", "selunet_gemm_wgrad", "selunet_gemm_wgrad_ws")

    def __init__(self, esz):
        self.active = False
        self.esz = esz
        self.rec = {}  # kernel name -> list of (start, end, flops, bytes)
        self.shapes = {}  # (kernel name, operand shape) -> list of (start, end, flops)

    @staticmethod
    def _k(g):
        return g.taps * sum(g.src[i].channels for i in range(g.nsrc))

    def _src_bytes(self, g):
        hs, ws = (2 * g.h, 2 * g.w) if g.taps == 4 else (g.h, g.w)
        return sum(g.n * hs * ws * g.src[i].channels * (4 if g.src[i].layout == 1 else self.esz)
                   for i in range(g.nsrc))

    def __call__(self, name, args, fn):
        if not self.active or name not in self.ENTRY:
            return fn()
        if name == "selunet_gemm_gather":
            g, n_cols, mode = args[0], args[2], args[4].mode
            kname = K.query("selunet_gemm_kernel_name", g, None, n_cols, mode, args[5]).decode()
            m = g.n * g.h * g.w
            flops = 2.0 * m * n_cols * self._k(g)
            nbytes = self._src_bytes(g) + m * n_cols * self.esz + n_cols * self._k(g) * self.esz
            shape = f"gather {g.h}x{g.w} taps={g.taps} K={self._k(g)} N={n_cols} mode={mode}"
        else:
            gp, gq = args[0], args[1]
            dt = args[3] if name == "selunet_gemm_wgrad" else args[5]
            kname = K.query("selunet_gemm_kernel_name", gp, gq, 0, 0, dt).decode()
            if name == "selunet_gemm_wgrad_ws" and args[4] > 0:
                kname += "+reduce"  # (the entry point's time includes the split reduction)
            flops = 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)
            nbytes = self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            shape = f"wgrad {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}"
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn()
        e.record()
        self.rec.setdefault(kname, []).append((s, e, flops, nbytes))
        self.shapes.setdefault((kname, shape), []).append((s, e, flops))
        return rc

    def shape_summary(self, steps):
        rows = []
        for (k, shape), lst in self.shapes.items():
            ms = sum(s.elapsed_time(e) for s, e, _ in lst)
            fl = sum(f for _, _, f in lst)
            rows.append((ms / steps, k, shape, len(lst) // steps, fl / (ms * 1e-3) / 1e12 if ms else 0.0))
        return sorted(rows, reverse=True)

    def summary(self):
        out = {}
        for k, lst in self.rec.items():
            out[k] = {"ms": sum(s.elapsed_time(e) for s, e, _, _ in lst), "launches": len(lst),
                      "flops": sum(f for _, _, f, _ in lst), "bytes": sum(b for _, _, _, b in lst)}
        return out


def load_traffic(kernel):
    """PMC-measured HBM bytes per launch for `kernel` from the committed profile summary
    (profiles/*_traffic.json, written by tools/pmc_summary.py --traffic), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if kernel in d.get("kernels", {}):
            return d["kernels"][kernel], os.path.relpath(path, REPO)
    return None, None


def cpu_baseline(args):
    """Time the CPU oracle (reference op sequence, torch eager fp32) on a bounded sample."""
    from oracle import unet_b_cpu as O

    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cores = max(1, min(cores, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    x, lab = make_batch(args.cpu_batch, args.size, seed=123)
    xt, lt = torch.tensor(x), torch.tensor(lab)
    params, buffers = O.make_state(0, "RGB", True)
    opt = O.AdamRef(params.values(), lr=1e-3)
    O.train_step(params, buffers, opt, xt, lt, True, lamb=args.lamb)  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        O.train_step(params, buffers, opt, xt, lt, True, lamb=args.lamb)
    dt = time.perf_counter() - t0
    return {"value": round(args.cpu_batch * args.cpu_steps / dt, 4), "unit": "images/s", "cores": cores,
            "kind": "port",
            "sample": f"{args.cpu_steps} timed steps (+1 warm-up) of the oracle train step, SelectiveUNet_B "
                      f"bs={args.cpu_batch} {args.size}x{args.size} fp32, torch {torch.__version__} CPU, "
                      f"{cores} threads; {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        parallel.init_data_parallel(backend="nccl")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    net = S.UNet_B("RGB", selective=True, compute_dtype=dt)
    p = L.seeded_params(0, "RGB", True, bn_affine_random=False)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(dev).train()
    parallel.broadcast_params(net)
    opt = S.Adam(net.parameters(), lr=1e-3)
    loss_a = S.BCEWithLogitsLoss()

    x, lab = make_batch(args.batch, args.size, seed=0)
    lo, hi = parallel.chunk_bounds(args.batch, rank, world)
    parallel.set_global_batch(args.batch)
    xt = torch.tensor(x[lo:hi], device=dev)
    lt = torch.tensor(lab[lo:hi], device=dev)
    del x, lab

    timer = KernelTimer(2 if dt == torch.bfloat16 else 4)
    # per-kernel HIP-event timing (the roofline object) at N = 1; multi-GPU lines skip it, so the
    # event records add no host work to the small per-GPU steps of the scaling runs
    if world > 1:
        args.no_kernel_timing = True
    if not args.no_kernel_timing:
        K.set_call_hook(timer)

    def step():
        out, sel, aux = net(xt)
        aux_loss = loss_a(aux, lt)
        sel_loss, cov = S.calc_selective_risk_image_b(out, sel, target=lt, lamb=args.lamb)
        loss = aux_loss + sel_loss
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timer.active = False
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())

    value = args.batch * args.steps / elapsed
    ms_step = 1e3 * elapsed / args.steps
    roof = None
    ksum = timer.summary() if not args.no_kernel_timing else None
    if ksum:
        dom = max(ksum, key=lambda n: ksum[n]["ms"])
        d = ksum[dom]
        peak, unit = PEAK[args.dtype]
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12 if d["ms"] > 0 else 0.0
        launches = max(1, d["launches"])
        # the committed PMC summary was collected on the default workload (bs=128 per GPU, 256x256);
        # its per-launch bytes describe other shapes' launches not at all
        traffic, tsrc = load_traffic(dom) if (args.size, hi - lo) == (256, 128) else (None, None)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4),
                "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
                "traffic_source": tsrc,
                "algorithmic_flops_per_launch": d["flops"] / launches,
                "algorithmic_bytes_per_launch": d["bytes"] / launches,
                "per_launch_ms": round(d["ms"] / launches, 4),
                "launches": d["launches"], "kernel_share_of_step": round(d["ms"] / (elapsed * 1e3), 4),
                "all": {n: {"ms_per_step": round(v["ms"] / args.steps, 3), "launches_per_step": v["launches"] // args.steps,
                            "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2) if v["ms"] else 0.0,
                            "hbm_gbs_algorithmic": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else 0.0}
                        for n, v in sorted(ksum.items(), key=lambda kv: -kv[1]["ms"])}}
        if args.layer_report and rank == 0:
            for ms, k, shape, n, tf in timer.shape_summary(args.steps):
                print(f"{ms:7.3f} ms/step {n:2d}x {tf:7.1f} TF/s  {k:26s} {shape}", file=sys.stderr)
    whole = TRAIN_GFLOP_PER_IMG_256 * (args.size / 256) ** 2 * value / 1e3  # TFLOP/s whole step
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        line = {
            "metric": f"train images/sec, SelectiveUNet_B {args.size}x{args.size} bs={args.batch} (global), "
                      f"selective_loss s_lamb={args.lamb:g}",
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic (seeded tumor/benign {args.size}x{args.size} patches, HBM-resident)",
            "config": {"workload": f"SelectiveUNet_B train step, global bs={args.batch}, {args.size}x{args.size}, "
                                   f"Adam lr=1e-3, s_lamb={args.lamb:g}", "model": "SelectiveUNet_B",
                       "global_batch": args.batch, "per_gpu_batch": hi - lo, "image": args.size,
                       "parallelism": f"dp{world}"},
            "step_tflops": round(whole, 2), "step_mfma_frac": round(whole / world / PEAK[args.dtype][0], 4),
            "final_loss": round(final_loss, 5),
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
