"""Time selunet_bn_bwd_apply at the bench shapes (bs=128 bf16) — profiling tool."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402

tot, byt = 0.0, 0
for c, r in ((64, 256), (128, 128), (256, 64), (512, 32)):
    m = 128 * r * r
    dz = torch.randn(m, c, device="cuda").bfloat16()
    y = torch.randn(m, c, device="cuda").bfloat16()
    dy = torch.empty_like(dz)
    v = [torch.rand(c, device="cuda") + 0.5 for _ in range(4)]
    coef = torch.randn(3, c, device="cuda")
    f = lambda: K.call("selunet_bn_bwd_apply", K.ptr(dz), K.ptr(y), m, c, *[K.ptr(t) for t in v], K.ptr(coef),  # noqa
                       K.ptr(dy), K.BF16, K.stream_ptr())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    tot += ms
    byt += 3 * m * c * 2
    print(f"C={c} @{r}: {ms:.3f} ms  {3 * m * c * 2 / ms / 1e6:.0f} GB/s", flush=True)
print(f"total {tot:.3f} ms  {byt / tot / 1e6:.0f} GB/s")
