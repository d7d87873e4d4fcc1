"""Benchmark: SelectiveUNet_B training images/sec, 256x256, global batch 128 (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]                       # N = 1
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N  # N > 1 (RCCL)

One step = the reference's training iteration (train.py:186-209) on synthetic, HBM-resident
data: forward of UNet_B(selective=True), BCEWithLogits aux loss + calc_selective_risk_image_b
(s_lamb=2), backward (with the RCCL gradient all-reduce when N > 1) and the Adam update. The
global batch of 128 is split into contiguous per-rank chunks (DataParallel semantics), so
`scaling` is "strong". Rank 0 prints one JSON line.

`value` is the fp32 configuration — the reference's arithmetic (model.py:9-15, train.py:194-209):
fp32 tensors, statistics, losses and optimizer, with the 3x3 and ConvTranspose2d contractions on
split-fp16 operands (each fp32 operand = fp16 high + low parts, 22 significant bits; three
v_mfma_f32_32x32x16_f16 products per fp32 product, fp32 accumulation) — timed with no
profiling hook installed. The same run then measures the step with every convolution on exact fp32
MFMA products (`exact_f32` key, v_mfma_f32_32x32x2_f32, SELUNET_X2=0) and the bf16 speed
configuration (`bf16` key) the same way. `step_mfma_frac` divides the step's direct-convolution
FLOP rate by the ceiling of the arithmetic actually run: fp16 dense peak / 3 for split-fp16, the
bf16 peak for `bf16` (none for `exact_f32`: its Winograd kernels execute 2/3 of the direct FLOPs).
For each configuration, after the headline timing:
  * `roofline`: a separate pass with every kernel entry point bracketed by HIP events on the
    launch stream; the dominant kernel's algorithmic FLOPs (MFMA-bound) or bytes (HBM-bound) per
    launch divided by its average launch duration, against the MI355X peak for its bound;
  * `full_loop`: the step plus the on-device train-loop metrics (train.py:211-241 restated:
    thresholded masks, confusion matrix, rejection counts, loss sums; metrics.SegMetrics), read
    back once at the end — SURVEY.md §8(d) timing (b).
`cpu_baseline` times the CPU oracle (oracle/unet_b_cpu.py, the reference's op sequence in torch
eager on the host cores) on a bounded sample.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import platform
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
from selectivenet_for_semantic_segmentation_binary_amd.metrics import SegMetrics  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402

TRAIN_GFLOP_PER_IMG_256 = 220.38  # fwd 73.535 x 3 - first-layer dgrad
PEAK = {"bf16": (2500.0, "TFLOP/s"), "fp32": (157.3, "TFLOP/s")}  # MI355X dense MFMA (MICROARCH guide)
# ceiling of one fp32 product on split-fp16 operands: three fp16 MFMA products each
X2_CEILING_TFLOPS = PEAK["bf16"][0] / 3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="global batch (split over ranks)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="fp32", help="headline configuration")
    ap.add_argument("--no-bf16", action="store_true", help="skip the extra bf16 measurement")
    ap.add_argument("--no-exact", action="store_true", help="skip the extra exact-fp32-MFMA measurement")
    ap.add_argument("--selective", type=int, default=1, help="0: non-selective UNet_B (BASELINE configs[1])")
    ap.add_argument("--lamb", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=3, help="steps of the per-kernel attribution pass")
    ap.add_argument("--no-full-loop", action="store_true")
    ap.add_argument("--no-input-loop", action="store_true", help="skip the timed loop fed by the patch loader")
    ap.add_argument("--layer-report", action="store_true", help="print per-entry-point timing to stderr")
    ap.add_argument("--no-size512", action="store_true",
                    help="skip the BASELINE configs[4] measurement (512x512, global bs=64, `size512` key)")
    return ap.parse_args()


def _i(v):
    return int(getattr(v, "value", v))


class KernelTimer:
    """Brackets the kernel entry points with HIP events on the launch stream (torch's current
    stream, the one the kernels are launched on) and attributes each launch to the kernel it
    dispatches to, with its algorithmic FLOPs (2*M*N*K of the true, unpadded GEMM) and algorithmic
    HBM bytes (each operand tensor read once, each output written once) and its bound."""

    MFMA = ("selunet_gemm_gather", "selunet_gemm_gather_x2", "selunet_conv3x3_wino", "selunet_conv3x3_x2",
            "selunet_conv3x3_wgrad_x2", "selunet_conv3x3_wgrad_x2_bn", "selunet_conv3x3_wgrad_x2_bn_src",
            "selunet_gemm_wgrad_x2",
            "selunet_gemm_wgrad", "selunet_gemm_wgrad_ws", "selunet_gemm_wgrad_ws_to")
    HBM = ("selunet_first_conv_fwd", "selunet_first_conv_fwd_centered", "selunet_first_conv_wgrad", "selunet_bn_bwd_apply", "selunet_bn_bwd_apply_amax",
           "selunet_maxpool2_fwd",
           "selunet_maxpool2_bwd", "selunet_heads_fwd", "selunet_heads_bwd", "selunet_bn_bwd_apply_heads",
           "selunet_bn_bwd_apply_pool", "selunet_bn_bwd_apply_heads_planes")

    def __init__(self, esz, tag):
        self.active = False
        self.esz = esz
        self.tag = tag
        self.rec = {}  # kernel name -> list of (start, end, flops, bytes)
        self.bound = {}
        self.shapes = {}  # (kernel name, operand shape) -> list of (start, end, flops)

    @staticmethod
    def _k(g):
        return g.taps * sum(g.src[i].channels for i in range(g.nsrc))

    def _src_bytes(self, g):
        hs, ws = (2 * g.h, 2 * g.w) if g.taps == 4 else (g.h, g.w)
        return sum(g.n * hs * ws * g.src[i].channels * (4 if g.src[i].layout == 1 else self.esz)
                   for i in range(g.nsrc))

    def _describe(self, name, args):
        esz, t = self.esz, self.tag
        if name == "selunet_gemm_gather":
            g, n_cols, mode = args[0], _i(args[2]), args[4].mode
            kname = K.query("selunet_gemm_kernel_name", g, None, n_cols, mode, _i(args[5])).decode()
            m = g.n * g.h * g.w
            flops = 2.0 * m * n_cols * self._k(g)
            nbytes = self._src_bytes(g) + m * n_cols * esz + n_cols * self._k(g) * esz
            return kname, "mfma", flops, nbytes, f"gather {g.h}x{g.w} taps={g.taps} K={self._k(g)} N={n_cols} mode={mode}"
        if name == "selunet_gemm_gather_x2":  # (g, w, n_cols, k_pad, ep, amax0, amax1, stream)
            g, n_cols, mode = args[0], _i(args[2]), args[4].mode
            m = g.n * g.h * g.w
            flops = 3 * 2.0 * m * n_cols * self._k(g)  # executed fp16 MFMA work
            nbytes = self._src_bytes(g) + m * n_cols * esz + n_cols * self._k(g) * esz
            return ("gemm_gather_x2<f32>", "mfma_f16", flops, nbytes,
                    f"gather x2 {g.h}x{g.w} taps={g.taps} K={self._k(g)} N={n_cols} mode={mode}")
        if name == "selunet_conv3x3_wino":  # (g, u, n_cols, ep, stream): fp32 Winograd F(2,3)
            g, n_cols, ep = args[0], _i(args[2]), args[3]
            kname = K.query("selunet_conv3x3_wino_kernel_name", n_cols, ep.mode, ep.split).decode()
            m = g.n * g.h * g.w
            c = self._k(g) // 9
            # the MFMA work the algorithm does: 12 (dy, xi) passes per output pair = 6 per pixel
            # (the direct 3x3 conv does 9; its FLOP count is 1.5x these)
            flops = 2.0 * m * n_cols * 6 * c
            nbytes = self._src_bytes(g) + m * n_cols * esz + n_cols * 12 * c * esz
            return kname, "mfma", flops, nbytes, f"wino {g.h}x{g.w} C={c} N={n_cols} mode={ep.mode}"
        if name == "selunet_conv3x3_x2":  # (g, w, n_cols, ep, amax0, amax1, stream): split-fp16 fp32 conv
            g, n_cols, ep = args[0], _i(args[2]), args[3]
            kname = K.query("selunet_conv3x3_x2_kernel_name", g, n_cols, ep.mode, ep.split).decode()
            m = g.n * g.h * g.w
            # the fp16 MFMA work executed: three products (hh, hl, lh) per fp32 product, against the
            # fp16 dense peak ("mfma_f16")
            flops = 3 * 2.0 * m * n_cols * self._k(g)
            nbytes = self._src_bytes(g) + m * n_cols * esz + n_cols * self._k(g) * esz
            return kname, "mfma_f16", flops, nbytes, f"x2 {g.h}x{g.w} K={self._k(g)} N={n_cols} mode={ep.mode}"
        if name == "selunet_conv3x3_wgrad_x2":  # (gp, gq, ws, wsb, out, amax_p, amax_q0, amax_q1, stream)
            gp, gq = args[0], args[1]
            kname = f"conv3x3_wgrad_x2<{128 if self._k(gp) % 128 == 0 else 64}>+reduce"
            flops = 3 * 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)  # executed fp16 MFMA work
            nbytes = self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            return kname, "mfma_f16", flops, nbytes, f"wgrad x2 {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}"
        if name == "selunet_conv3x3_wgrad_x2_bn":  # the BN-backward apply fused: reads dA and y, writes dy
            gp, gq = args[0], args[1]
            kname = f"conv3x3_wgrad_x2_bn<{128 if self._k(gp) % 128 == 0 else 64}>+reduce"
            flops = 3 * 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)
            nbytes = 3 * self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            return kname, "mfma_f16", flops, nbytes, f"wgrad x2 bn {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}"
        if name == "selunet_conv3x3_wgrad_x2_bn_src":  # the pool / heads applies fused (args[10]: the dA source)
            gp, gq, src = args[0], args[1], args[10]
            flops = 3 * 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)
            m = gp.n * gp.h * gp.w
            if src.kind == K.DA_POOL:  # reads y, skip and the pooled gradient, writes dy
                form, dab = "pool", (1 + (1 if src.skip else 0) + 0.25) * self._src_bytes(gp)
            else:  # reads y and the heads' gradient planes, writes dy
                form, dab = "heads", self._src_bytes(gp) + 4.0 * m * src.nh
            nbytes = dab + self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            return (f"conv3x3_wgrad_x2_{form}<{128 if self._k(gp) % 128 == 0 else 64}>+reduce", "mfma_f16", flops, nbytes,
                    f"wgrad x2 {form} {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}")
        if name == "selunet_gemm_wgrad_x2":  # (gp, gq, ws, wsb, layout, out, amax_p0, p1, q0, q1, stream)
            gp, gq = args[0], args[1]
            flops = 3 * 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)  # executed fp16 MFMA work
            nbytes = self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            return ("gemm_wgrad_x2<f32>+reduce", "mfma_f16", flops, nbytes,
                    f"wgrad gx2 {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}")
        if name in ("selunet_gemm_wgrad", "selunet_gemm_wgrad_ws", "selunet_gemm_wgrad_ws_to"):
            gp, gq = args[0], args[1]
            dt = _i(args[{"selunet_gemm_wgrad": 3, "selunet_gemm_wgrad_ws": 5, "selunet_gemm_wgrad_ws_to": 7}[name]])
            kname = K.query("selunet_gemm_kernel_name", gp, gq, 0, 0, dt).decode()
            if name != "selunet_gemm_wgrad" and _i(args[4]) > 0:
                kname += "+reduce"  # (the entry point's time includes the split reduction)
            flops = 2.0 * gp.n * gp.h * gp.w * self._k(gp) * self._k(gq)
            if "wino" in kname:  # Winograd F(2,3) transpose: 4 products per output pair and row, not 6
                flops *= 2.0 / 3.0
            nbytes = self._src_bytes(gp) + self._src_bytes(gq) + 4 * self._k(gp) * self._k(gq)
            return kname, "mfma", flops, nbytes, f"wgrad {gp.h}x{gp.w} Kp={self._k(gp)} Kq={self._k(gq)}"
        if name in ("selunet_first_conv_fwd", "selunet_first_conv_fwd_centered"):  # (x, n, cin, h, w, wpack, y, ...)
            n, cin, h, w = (_i(a) for a in args[1:5])
            m = n * h * w
            return (f"first_conv_fwd<{t}>", "hbm", 2.0 * m * 64 * 9 * cin, m * cin * 4 + m * 64 * esz,
                    f"first fwd {h}x{w}")
        if name == "selunet_first_conv_wgrad":  # (x, n, cin, h, w, dy, slab, dtype, stream)
            n, cin, h, w = (_i(a) for a in args[1:5])
            m = n * h * w
            return (f"first_conv_wgrad<{t}>", "hbm", 2.0 * m * 64 * 9 * cin, m * cin * 4 + m * 64 * esz,
                    f"first wgrad {h}x{w}")
        if name in ("selunet_bn_bwd_apply", "selunet_bn_bwd_apply_amax"):  # (dA, y, M, C, ...): read dA + y, write dy
            m, c = _i(args[2]), _i(args[3])
            return f"bn_bwd_apply<{t}>", "hbm", 0.0, 3 * m * c * esz, f"bn_bwd_apply C={c}"
        if name == "selunet_maxpool2_fwd":  # (y, n, h, w, c, ...): read y, write y/4
            n, h, w, c = (_i(a) for a in args[1:5])
            return f"maxpool2_fwd<{t}>", "hbm", 0.0, 1.25 * n * h * w * c * esz, f"pool fwd {h}x{w} C={c}"
        if name == "selunet_maxpool2_bwd":  # (y, n, h, w, c, sc, sh, dp, dskip, dz, ...)
            n, h, w, c = (_i(a) for a in args[1:5])
            m = n * h * w
            skip = args[8] is not None and _i(args[8]) != 0
            wr = args[9] is not None and _i(args[9]) != 0  # (dz null: the BN-backward sums only)
            return (f"maxpool2_bwd<{t}>", "hbm", 0.0, (1.25 + (1 if wr else 0) + (1 if skip else 0)) * m * c * esz,
                    f"pool bwd {h}x{w} C={c}")
        if name == "selunet_heads_fwd":  # (y, M, sc, sh, w, b, nheads, o0, o1, o2, ...)
            m, nh = _i(args[1]), _i(args[6])
            return f"heads_fwd<{t}>", "hbm", 2.0 * m * 64 * nh, m * 64 * esz + nh * m * 4, "heads fwd"
        if name == "selunet_heads_bwd":  # (y, M, sc, sh, w, nheads, g0, g1, g2, dz, ...)
            m, nh = _i(args[1]), _i(args[5])
            wr = args[9] is not None and _i(args[9]) != 0  # (dz null: the sums only)
            return (f"heads_bwd<{t}>", "hbm", 4.0 * m * 64 * nh, (2 if wr else 1) * m * 64 * esz + nh * m * 4,
                    "heads bwd")
        if name == "selunet_bn_bwd_apply_heads":  # (y, M, sc, sh, mean, invstd, coef, w, nh, g0, g1, g2, dy, ...)
            m, nh = _i(args[1]), _i(args[8])
            return f"bn_bwd_apply<{t}>", "hbm", 0.0, 2 * m * 64 * esz + nh * m * 4, "bn_bwd_apply heads"
        if name == "selunet_bn_bwd_apply_heads_planes":  # (y, M, sc, sh, mean, invstd, coef, w, planes, dy, ...)
            m, nk = _i(args[1]), int(args[8].n)
            return f"bn_bwd_apply<{t}>", "hbm", 0.0, 2 * m * 64 * esz + nk * m * 4, "bn_bwd_apply heads planes"
        if name == "selunet_bn_bwd_apply_pool":  # (y, n, h, w, c, sc, sh, mean, invstd, coef, dp, dskip, dy, ...)
            n, h, w, c = (_i(a) for a in args[1:5])
            m = n * h * w
            skip = args[11] is not None and _i(args[11]) != 0
            return (f"bn_bwd_apply<{t}>", "hbm", 0.0, (2.25 + (1 if skip else 0)) * m * c * esz,
                    f"bn_bwd_apply pool {h}x{w} C={c}")
        return None

    def __call__(self, name, args, fn):
        if not self.active or (name not in self.MFMA and name not in self.HBM):
            return fn()
        kname, bound, flops, nbytes, shape = self._describe(name, args)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn()
        e.record()
        self.bound[kname] = bound
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
                      "flops": sum(f for _, _, f, _ in lst), "bytes": sum(b for _, _, _, b in lst),
                      "bound": self.bound[k]}
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


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
            "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{args.cpu_steps} timed steps (+1 warm-up) of the oracle train step, SelectiveUNet_B "
                      f"bs={args.cpu_batch} {args.size}x{args.size} fp32, torch {torch.__version__} CPU, "
                      f"{cores} threads of {cpu_model()}; {dt:.1f} s"}


def timed(fn, steps, world, dev):
    """Run fn `steps` times between barrier + synchronize brackets; max over ranks (seconds)."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def run_config(args, dtype, world, rank, dev, xt, lt, local_batch):
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    selective = bool(args.selective)
    net = S.UNet_B("RGB", selective=selective, compute_dtype=dt)
    p = L.seeded_params(0, "RGB", selective, bn_affine_random=False)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(dev).train()
    parallel.broadcast_params(net)
    opt = S.Adam(net.parameters(), lr=1e-3)
    loss_a = S.BCEWithLogitsLoss()
    state = {}

    def step(x=xt, t=lt):
        if selective:
            out, sel, aux = net(x)
            loss = loss_a(aux, t)
            sel_loss, _ = S.calc_selective_risk_image_b(out, sel, target=t, lamb=args.lamb)
            loss = loss + sel_loss
        else:
            out, sel = net(x), None
            loss = loss_a(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        state["loss"], state["out"], state["sel"] = loss, out, sel
        return loss

    for _ in range(args.warmup):
        step()
    elapsed = timed(step, args.steps, world, dev)
    final_loss = float(state["loss"].item())
    res = {"value": round(args.batch * args.steps / elapsed, 2), "ms_per_step": round(1e3 * elapsed / args.steps, 3),
           "final_loss": round(final_loss, 5)}

    # per-kernel attribution: its own pass, so the headline steps carry no event records
    if not args.no_kernel_timing:
        timer = KernelTimer(2 if dt == torch.bfloat16 else 4, "bf16" if dt == torch.bfloat16 else "f32")
        K.set_call_hook(timer)
        timer.active = True
        ksteps = max(1, args.kernel_steps)
        kel = timed(step, ksteps, world, dev)
        timer.active = False
        K.set_call_hook(None)
        res["roofline"] = roofline(args, dtype, timer, ksteps, kel, local_batch)
        if args.layer_report and rank == 0:
            for ms, k, shape, n, tf in timer.shape_summary(ksteps):
                print(f"[{dtype}] {ms:7.3f} ms/step {n:2d}x {tf:7.1f} TF/s  {k:30s} {shape}", file=sys.stderr)

    # full training-loop iteration: step + on-device metrics and loss sums (train.py:194-241)
    if not args.no_full_loop:
        ev = SegMetrics(dev, selective=selective, rule="train")
        sums = torch.zeros(3, dtype=torch.float64, device=dev)

        def loop_step():
            loss = step()
            sums[0] += loss.detach()
            ev.add_batch(state["out"].detach(), lt, None if state["sel"] is None else state["sel"].detach())

        def loop(nsteps):
            for _ in range(nsteps):
                loop_step()
            ev.raw()  # the per-epoch read-back (all-reduced over ranks)
            sums.cpu()

        loop(1)
        el = timed(lambda: loop(args.steps), 1, world, dev)
        res["full_loop"] = {"value": round(args.batch * args.steps / el, 2), "ms_per_step": round(1e3 * el / args.steps, 3),
                            "includes": "step + SegMetrics.add_batch (thresholded masks, 2x2 confusion matrix, "
                                        "rejection counts) + loss sums, read back once"}
        if not args.no_input_loop and world == 1 and dtype == args.dtype:
            res["input_loop"] = input_loop(args, dev, step, state, selective)
    res["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    del net, opt, state, step
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    return res


def input_loop(args, dev, step, state, selective):
    """The training loop fed by the patch loader instead of HBM-resident tensors (train.py:183-191 +
    utils/data_utils.py:200-236 restated): data.BatchLoader gathers each shuffled global batch of
    uint8 NHWC patches into pinned host memory on a prefetch thread, copies it to the GPU (uint8:
    4x fewer bytes than the reference's fp32 input) and expands it there (selunet_prep_batch_mode:
    /255, Normalization, RandomFlip, NCHW fp32, label truncation); then the step and the on-device
    metrics. Synthetic patches (2 global batches, cycled over epochs). Also times the reference's
    own per-step input copy, the pageable fp32 [B,3,H,W] tensor .to(cuda) of train.py:186."""
    from selectivenet_for_semantic_segmentation_binary_amd import data as D

    ds = D.synthetic_patchset(2 * args.batch, args.size, seed=5)
    loader = D.BatchLoader(ds, args.batch, shuffle=True, random_flip=True, device=dev)
    ev = SegMetrics(dev, selective=selective, rule="train")
    epoch = [0]

    def run(nsteps):
        done = 0
        while done < nsteps:
            loader.set_epoch(epoch[0])
            epoch[0] += 1
            for x, t in loader:
                step(x, t)
                ev.add_batch(state["out"].detach(), t, None if state["sel"] is None else state["sel"].detach())
                done += 1
                if done == nsteps:
                    break
        ev.raw()

    run(2)
    el = timed(lambda: run(args.steps), 1, 1, dev)
    # the reference's input copy: pageable fp32 NCHW batch -> GPU (train.py:186)
    xh = torch.empty(args.batch, 3, args.size, args.size, dtype=torch.float32)
    xh.fill_(0.5)
    xh.to(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        xh.to(dev)
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t0) / 5
    return {"value": round(args.batch * args.steps / el, 2), "ms_per_step": round(1e3 * el / args.steps, 3),
            "includes": "data.BatchLoader (shuffled uint8 NHWC patches gathered into pinned memory on a prefetch "
                        "thread, H2D copy as uint8 on a copy stream overlapping the previous step, GPU normalise / "
                        "flips / NCHW fp32) + step + SegMetrics",
            "reference_fp32_h2d_ms": round(1e3 * h2d, 3),
            "reference_fp32_h2d_note": f"pageable fp32 [{args.batch},3,{args.size},{args.size}] .to(cuda) per step "
                                       f"(train.py:186), {xh.numel() * 4 / 1e6:.1f} MB; not in any timed value"}


def roofline(args, dtype, timer, ksteps, kel, local_batch):
    ksum = timer.summary()
    if not ksum:
        return None
    mfma_peak, mfma_unit = PEAK[dtype]

    def frac(v):
        if v["ms"] <= 0:
            return 0.0, 0.0
        if v["bound"] in ("mfma", "mfma_f16"):
            a = v["flops"] / (v["ms"] * 1e-3) / 1e12
            return a, a / (PEAK["bf16"][0] if v["bound"] == "mfma_f16" else mfma_peak)
        a = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        return a, a / HBM_PEAK_GBS

    dom = max(ksum, key=lambda n: ksum[n]["ms"])
    d = ksum[dom]
    achieved, fr = frac(d)
    launches = max(1, d["launches"])
    # the committed PMC summary was collected on the default workload (bs=128 per GPU, 256x256)
    traffic, tsrc = load_traffic(dom) if (args.size, local_batch) == (256, 128) else (None, None)
    hbm = d["bound"] == "hbm"
    f16 = d["bound"] == "mfma_f16"
    return {
        "bound": "mfma" if f16 else d["bound"], "kernel": dom, "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS if hbm else (PEAK["bf16"][0] if f16 else mfma_peak),
        "unit": "GB/s" if hbm else mfma_unit, "frac": round(fr, 4),
        "peak_basis": "fp16 dense MFMA peak; achieved counts the three fp16 products per fp32 product the "
                      "split-fp16 kernel executes" if f16 else None,
        "traffic": traffic["hbm_bytes_per_launch"] if traffic else None, "traffic_source": tsrc,
        "algorithmic_flops_per_launch": d["flops"] / launches, "algorithmic_bytes_per_launch": d["bytes"] / launches,
        "per_launch_ms": round(d["ms"] / launches, 4), "launches": d["launches"],
        "kernel_share_of_step": round(d["ms"] / (kel * 1e3), 4),
        "timing": f"HIP events on the launch stream, separate {ksteps}-step pass after the headline timing",
        "all": {n: {"bound": v["bound"], "ms_per_step": round(v["ms"] / ksteps, 3),
                    "launches_per_step": v["launches"] // ksteps,
                    "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2) if v["ms"] else 0.0,
                    "hbm_gbs_algorithmic": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else 0.0,
                    "frac": round(frac(v)[1], 4)}
                for n, v in sorted(ksum.items(), key=lambda kv: -kv[1]["ms"])},
    }


def run_size512(args, world, rank, dev):
    """BASELINE configs[4]: SelectiveUNet_B on 512x512 patches, global bs=64 split over the ranks as
    the headline splits its 128 (DataParallel chunks), the same fp32 configuration and the same
    barrier-bracketed max-over-ranks timing; the step alone (no per-kernel or loop passes)."""
    import copy
    a = copy.copy(args)
    a.size, a.batch = 512, 64
    a.no_kernel_timing = a.no_full_loop = a.no_input_loop = True
    x, lab = make_batch(a.batch, a.size, seed=0)
    lo, hi = parallel.chunk_bounds(a.batch, rank, world)
    parallel.set_global_batch(a.batch)
    xt = torch.tensor(x[lo:hi], device=dev)
    lt = torch.tensor(lab[lo:hi], device=dev)
    del x, lab
    try:
        r = run_config(a, args.dtype, world, rank, dev, xt, lt, hi - lo)
    finally:
        parallel.set_global_batch(args.batch)
    r.pop("full_loop", None)
    r["config"] = {"workload": f"SelectiveUNet_B train step, global bs=64, 512x512, Adam lr=1e-3, s_lamb={a.lamb:g}",
                   "global_batch": 64, "per_gpu_batch": hi - lo, "image": 512, "parallelism": f"dp{world}"}
    r["unit"] = "images/s"
    r["step_tflops"] = round(TRAIN_GFLOP_PER_IMG_256 * 4 * r["value"] / 1e3, 2)
    return r


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # (rehearsal of the N > 1 path on a one-GPU box: SELUNET_BENCH_ONE_DEVICE=1 puts every rank on
    # cuda:0 and uses gloo, which RCCL cannot; the driver's multi-GPU runs use one GPU per rank, RCCL)
    one_dev = os.environ.get("SELUNET_BENCH_ONE_DEVICE", "0") == "1"
    if one_dev:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        parallel.init_data_parallel(backend="gloo" if one_dev else "nccl")
        # the per-kernel event records add host work to the small per-GPU steps of the scaling runs
        args.no_kernel_timing = True

    x, lab = make_batch(args.batch, args.size, seed=0)
    lo, hi = parallel.chunk_bounds(args.batch, rank, world)
    parallel.set_global_batch(args.batch)
    xt = torch.tensor(x[lo:hi], device=dev)
    lt = torch.tensor(lab[lo:hi], device=dev)
    del x, lab

    head = run_config(args, args.dtype, world, rank, dev, xt, lt, hi - lo)
    extra = exact = None
    if args.dtype == "fp32" and not args.no_exact and world == 1:
        # the same fp32 step on the exact-fp32-MFMA kernels (Winograd / direct), for comparison
        os.environ["SELUNET_X2"] = "0"
        try:
            exact = run_config(args, "fp32", world, rank, dev, xt, lt, hi - lo)
        finally:
            os.environ.pop("SELUNET_X2", None)
    if args.dtype == "fp32" and not args.no_bf16:
        extra = run_config(args, "bf16", world, rank, dev, xt, lt, hi - lo)
    nosel = None
    if args.dtype == "fp32" and not args.no_bf16 and args.selective:
        # BASELINE configs[1]: UNet_B --selective 0 (the plain model, BCEWithLogits on its one head,
        # train.py:194-209 with selective off), the same global batch, bf16 — timed like the headline
        import copy
        a = copy.copy(args)
        a.selective = 0
        a.no_full_loop = a.no_input_loop = True
        nosel = run_config(a, "bf16", world, rank, dev, xt, lt, hi - lo)
        nosel["config"] = {"workload": f"UNet_B (selective 0) train step, global bs={args.batch}, "
                                       f"{args.size}x{args.size}, BCEWithLogits, Adam lr=1e-3",
                           "model": "UNet_B", "global_batch": args.batch, "per_gpu_batch": hi - lo,
                           "image": args.size, "parallelism": f"dp{world}"}
        nosel["unit"] = "images/s"
        nosel["note"] = ("BASELINE configs[1]: bf16 operands, fp32 accumulation and statistics; parity: "
                         "step_nosel_n128_256.npz [bf16] (tests/test_gpu_fullsize.py)")
    size512 = None
    if not args.no_size512 and (args.size, args.batch) == (256, 128):
        size512 = run_size512(args, world, rank, dev)
    group = None
    if world > 1:
        # the group every rank ran in, as torch.distributed reports it on that rank
        ws = torch.tensor([dist.get_world_size()], dtype=torch.int64, device=dev)
        lo_ws, hi_ws = ws.clone(), ws.clone()
        dist.all_reduce(lo_ws, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi_ws, op=dist.ReduceOp.MAX)
        group = {"backend": str(dist.get_backend()), "world_size": int(ws.item()),
                 "world_size_min_over_ranks": int(lo_ws.item()), "world_size_max_over_ranks": int(hi_ws.item()),
                 "rccl": str(dist.get_backend()) == "nccl" and torch.version.hip is not None}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        value = head["value"]
        whole = TRAIN_GFLOP_PER_IMG_256 * (args.size / 256) ** 2 * value / 1e3  # TFLOP/s whole step
        model = "SelectiveUNet_B" if args.selective else "UNet_B"
        what = f"selective_loss s_lamb={args.lamb:g}" if args.selective else "BCEWithLogits"
        line = {
            "metric": f"train images/sec, {model} {args.size}x{args.size} bs={args.batch} (global), {what}",
            "value": value, "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32" if args.dtype == "fp32" else "bf16",
            "data": f"synthetic (seeded tumor/benign {args.size}x{args.size} patches, HBM-resident)",
            "config": {"workload": f"{model} train step, global bs={args.batch}, {args.size}x{args.size}, "
                                   f"Adam lr=1e-3" + (f", s_lamb={args.lamb:g}" if args.selective else ""),
                       "model": model, "global_batch": args.batch, "per_gpu_batch": hi - lo, "image": args.size,
                       "parallelism": f"dp{world}",
                       "arithmetic": "fp32 tensors and accumulation; 3x3 forward and data-gradient convolutions "
                                     "on split-fp16 operands (each fp32 operand scaled by a power of two and "
                                     "split into fp16 high + low parts, 22 significant bits; three fp16 MFMA "
                                     "products per fp32 product; error vs fp64 at or below the exact fp32 MFMA's, "
                                     "tools/split_probe.hip), weight gradients likewise"
                       if args.dtype == "fp32" else "bf16 operands, fp32 accumulation"},
            "gpu": torch.cuda.get_device_name(dev),
            "step_tflops": round(whole, 2),
            "step_mfma_frac": round(whole / world / (X2_CEILING_TFLOPS if args.dtype == "fp32" else PEAK["bf16"][0]), 4),
            "step_flops_basis": "direct-convolution FLOPs of the training step; ceiling " + (
                "fp16 dense peak / 3 (split-fp16: three fp16 products per fp32 product)" if args.dtype == "fp32"
                else "bf16 dense peak"),
            "final_loss": head["final_loss"], "peak_hbm_gb": head["peak_hbm_gb"],
            "full_loop": head.get("full_loop"), "input_loop": head.get("input_loop"),
            "roofline": head.get("roofline"), "cpu_baseline": cpu,
            "process_group": group,
        }
        if size512 is not None:
            line["size512"] = size512
        if exact is not None:
            we = TRAIN_GFLOP_PER_IMG_256 * (args.size / 256) ** 2 * exact["value"] / 1e3
            # (direct-convolution FLOPs: the 1-D Winograd kernels execute 2/3 of them, so no fraction
            # of the fp32 MFMA peak is quoted for the whole step; roofline.all has each kernel's)
            exact["step_tflops_direct_equivalent"] = round(we, 2)
            exact["note"] = ("the same fp32 step with every convolution on exact fp32 MFMA products (1-D Winograd "
                             "F(2,3) forward / data-gradient / weight-gradient kernels; SELUNET_X2=0)")
            line["exact_f32"] = exact
        if extra is not None:
            wb = TRAIN_GFLOP_PER_IMG_256 * (args.size / 256) ** 2 * extra["value"] / 1e3
            extra["step_tflops"] = round(wb, 2)
            extra["step_mfma_frac"] = round(wb / world / PEAK["bf16"][0], 4)
            extra["note"] = "bf16 speed configuration (bf16 operands, fp32 accumulation); parity gates in DESIGN.md §4"
            line["bf16"] = extra
        if nosel is not None:
            line["bf16_nosel"] = nosel
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
