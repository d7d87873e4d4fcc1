"""Time the ConvTranspose2d GEMMs (selunet_gemm_gather SCATTER2X forward, taps=4 dgrad) at the
bench shapes (bs=128, bf16; --x2: the fp32 split-fp16 kernels and the weight gradient) — profiling tool, like tools/conv_bench.py.

    python tools/convt_bench.py [--batch 128] [--iters 10] [--x2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402

UPS = [("unpool3", 512, 256, 32), ("unpool2", 256, 128, 64), ("unpool1", 128, 64, 128)]  # name, Ci, Co, in-res


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--x2", action="store_true")
    a = ap.parse_args()
    n, dev = a.batch, "cuda"
    dt = torch.float32 if a.x2 else torch.bfloat16
    amax = torch.full((1,), 8.0, device=dev)
    tot = 0.0
    for name, ci, co, r in UPS:
        x = torch.randn(n * r * r, ci, device=dev).to(dt)
        sc, sh = torch.rand(ci, device=dev) + 0.5, torch.randn(ci, device=dev) * 0.1
        w = (torch.randn(4 * co * ci + 4 * co, device=dev).abs() * 1e-3 + 1e-3) if a.x2 else \
            (torch.randn(4 * co, ci, device=dev) * 0.05).to(dt)
        bias = torch.randn(co, device=dev)
        out = torch.empty(n * 4 * r * r, co, device=dev, dtype=dt)
        g = K.gather(n, r, r, 1, K.source(x, ci, sc, sh))
        ep = K.Epilogue(K.ptr(out), None, K.ptr(bias), None, K.EP_SCATTER2X, 0)
        amo = torch.zeros(1, device=dev)
        if a.x2:
            ep.amax = K.ptr(amo)  # the up-sampled tensor's range word, as in the step
        if a.x2:
            f = lambda: K.call("selunet_gemm_gather_x2", g, K.ptr(w), 4 * co, ci, ep, K.ptr(amax), None,  # noqa: E731
                               K.stream_ptr())
        else:
            f = lambda: K.call("selunet_gemm_gather", g, K.ptr(w), 4 * co, ci, ep, K.BF16, K.stream_ptr())  # noqa: E731
        ms = timed(f, a.iters)
        byt = (x.numel() + out.numel()) * x.element_size()
        tot += ms
        print(f"fwd   {name} {ci}->{co} @{r}: {ms:.3f} ms  {2 * n * r * r * ci * 4 * co / ms / 1e9:7.1f} TF/s "
              f"{byt / ms / 1e6:7.1f} GB/s", flush=True)
        du = torch.randn(n * 4 * r * r, co, device=dev).to(dt)
        wd = (torch.randn(ci * 4 * co + ci, device=dev).abs() * 1e-3 + 1e-3) if a.x2 else \
            (torch.randn(ci, 4 * co, device=dev) * 0.05).to(dt)
        dz = torch.empty(n * r * r, ci, device=dev, dtype=dt)
        gd = K.gather(n, r, r, 4, K.source(du, co))
        epd = K.Epilogue(K.ptr(dz), None, None, None, K.EP_PLAIN, 0)
        if a.x2:  # as in the training step: the BN-backward sums of the producer layer in the epilogue
            yprev = torch.randn(n * r * r, ci, device=dev)
            bn_c = [torch.rand(ci, device=dev) + 0.5 for _ in range(4)]
            rows = K.query("selunet_gemm_gather_x2_stats_rows", gd, ci)
            slab = torch.empty(rows, 3, ci, device=dev)
            epd.bnb = K.BnBwdStats(K.ptr(yprev), *(K.ptr(t) for t in bn_c), K.ptr(slab))
        if a.x2:
            fd = lambda: K.call("selunet_gemm_gather_x2", gd, K.ptr(wd), ci, 4 * co, epd, K.ptr(amax), None,  # noqa: E731
                                K.stream_ptr())
        else:
            fd = lambda: K.call("selunet_gemm_gather", gd, K.ptr(wd), ci, 4 * co, epd, K.BF16, K.stream_ptr())  # noqa: E731
        ms = timed(fd, a.iters)
        byt = (du.numel() + dz.numel()) * du.element_size()
        tot += ms
        print(f"dgrad {name} {co}->{ci} @{r}: {ms:.3f} ms  {2 * n * r * r * ci * 4 * co / ms / 1e9:7.1f} TF/s "
              f"{byt / ms / 1e6:7.1f} GB/s", flush=True)
        if a.x2:  # weight gradient: P = the layer input (BN+ReLU of its producer), Q = dU gathered per 2x2 tap
            gp = K.gather(n, r, r, 1, K.source(x, ci, sc, sh))
            gq = K.gather(n, r, r, 4, K.source(du, co))
            wsb = K.query("selunet_gemm_wgrad_x2_ws_bytes", gp, gq)
            ws = torch.empty(max(wsb // 4, 1), device=dev)
            gw = torch.empty(ci, co, 2, 2, device=dev)
            fw = lambda: K.call("selunet_gemm_wgrad_x2", gp, gq, K.ptr(ws), wsb, K.WG_CONVT, K.ptr(gw),  # noqa: E731
                                K.ptr(amax), None, K.ptr(amax), None, K.stream_ptr())
            ms = timed(fw, a.iters)
            byt = (x.numel() + du.numel()) * 4
            tot += ms
            print(f"wgrad {name} {ci}x{co}x4 @{r}: {ms:.3f} ms  {2 * n * r * r * ci * 4 * co / ms / 1e9:7.1f} TF/s "
                  f"{byt / ms / 1e6:7.1f} GB/s", flush=True)
    print(f"total {tot:.3f} ms")


if __name__ == "__main__":
    main()
