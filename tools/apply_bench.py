"""Time selunet_bn_bwd_apply(_amax) at the fp32 shapes of a batch (profiling tool).

    python tools/apply_bench.py [--iters 20] [--batch 128] [--forms 0,1,2,3] [--grids 1024]

--forms / --grids sweep SELUNET_OPT_APPLY_U8 (the kernel form) and SELUNET_OPT_APPLY_GRID (grid cap).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402

SHAPES = [(256 * 256, 64), (128 * 128, 128), (64 * 64, 256), (32 * 32, 512)]  # pixels per image, C


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--forms", default="0")
    ap.add_argument("--grids", default="1024")
    a = ap.parse_args()
    for form in [int(x) for x in a.forms.split(",")]:
        for grid in [int(x) for x in a.grids.split(",")]:
            K.set_option("APPLY_U8", form)
            K.set_option("APPLY_GRID", grid)
            print(f"form {form} grid {grid}", flush=True)
            run(a)


def run(a):
    tot = 0.0
    for px, c in SHAPES:
        m = a.batch * px
        dz, y = torch.randn(m, c, device="cuda"), torch.randn(m, c, device="cuda")
        dy = torch.empty_like(dz)
        co = [torch.rand(c, device="cuda") + 0.5 for _ in range(4)] + [torch.randn(3 * c, device="cuda")]
        amax = torch.zeros(1, device="cuda")

        def f():
            K.call("selunet_bn_bwd_apply_amax", K.ptr(dz), K.ptr(y), m, c, *[K.ptr(t) for t in co], K.ptr(dy),
                   K.ptr(amax), K.F32, K.stream_ptr())
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
        tot += ms
        print(f"apply m={m:9d} C={c:3d}: {ms:.3f} ms  {3 * m * c * 4 / ms / 1e9:7.2f} TB/s", flush=True)
    print(f"total {tot:.3f} ms")


if __name__ == "__main__":
    main()
