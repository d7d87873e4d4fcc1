"""Time the first layer's fused weight gradient (selunet_first_conv_wgrad_bn: encoder_layer_1_1's BN-backward
apply formed while staging, 3 -> 64 channels) at the bench shape (bs=128, 256x256, fp32) — profiling tool.

    python tools/first_bench.py [--batch 128] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n, h, w, dev = a.batch, 256, 256, "cuda"
    x = torch.randn(n, 3, h, w, device=dev)
    dz = torch.randn(n * h * w, 64, device=dev)
    y = torch.randn(n * h * w, 64, device=dev)
    c = [torch.rand(64, device=dev) + 0.5 for _ in range(4)]
    coef = torch.randn(3, 64, device=dev) * 1e-3
    rows = K.query("selunet_first_conv_wgrad_rows", n, h, w)
    slab = torch.empty(rows, 64, 32, device=dev)
    f = lambda: K.call("selunet_first_conv_wgrad_bn", K.ptr(x), n, 3, h, w, K.ptr(dz), K.ptr(y),  # noqa: E731
                       *(K.ptr(t) for t in c), K.ptr(coef), K.ptr(slab), K.F32, K.stream_ptr())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    byt = (dz.numel() + y.numel() + x.numel()) * 4
    print(f"first_conv_wgrad_bn bs={n}: {ms:.3f} ms  {byt / ms / 1e6:.1f} GB/s (dA + y + x read once)", flush=True)


if __name__ == "__main__":
    main()
