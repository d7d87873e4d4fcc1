"""Locate Winograd-kernel errors (debugging tool): per-pixel max error map of one case."""
import sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K  # noqa: E402
from tests.test_gpu_wino import pack_wino, gen, nhwc, nchw  # noqa: E402

def case(cin0, cin1, cout, n, h, w, xform, wgs):
    K.query("selunet_set_halo_workgroups", wgs)
    x0 = gen(n, cin0, h, w, seed=1)
    wt = gen(cout, cin0 + cin1, 3, 3, seed=3, scale=0.05)
    a = x0
    x0d = nhwc(x0).cuda()
    srcs = [K.source(x0d, cin0)]
    keep = [x0d]
    if cin1:
        x1 = gen(n, cin1, h, w, seed=2)
        a = torch.cat((a, x1), 1)
        x1d = nhwc(x1).cuda()
        keep.append(x1d)
        srcs.append(K.source(x1d, cin1))
    ref = F.conv2d(a.double(), wt.double(), padding=1)
    u, _ = pack_wino(wt, dgrad=False)
    y = torch.zeros(n * h * w, cout, device="cuda")
    g = K.gather(n, h, w, 9, *srcs)
    ep = K.Epilogue(K.ptr(y), None, None, None, K.EP_PLAIN, 0)
    res = []
    for it in range(3):
        K.call("selunet_conv3x3_wino", g, K.ptr(u), cout, ep, K.stream_ptr())
        torch.cuda.synchronize()
        got = nchw(y.cpu(), n, h, w).double()
        err = (got - ref).abs().amax(1) / ref.abs().max()   # [n,h,w]
        res.append(float(err.max()))
    print(f"case {cin0}+{cin1}->{cout} {n}x{h}x{w} wgs={wgs}: max err per run {res}")
    bad = (err > 1e-4).nonzero()
    if len(bad):
        ys = sorted(set(bad[:, 1].tolist())); xs = sorted(set(bad[:, 2].tolist()))
        print("  bad images", sorted(set(bad[:, 0].tolist())), "rows", ys[:40], "cols", xs[:40], "count", len(bad))
        cerr = (got - ref).abs().amax((0, 2, 3)) / ref.abs().max()
        print("  bad channels", (cerr > 1e-4).nonzero().flatten().tolist()[:64])

for c in [(64, 64, 128, 1, 16, 48, False, 0), (128, 0, 128, 1, 16, 48, False, 0), (64, 64, 128, 1, 16, 16, False, 0),
          (256, 0, 128, 2, 20, 24, False, 0), (256, 0, 128, 2, 32, 32, False, 0), (256, 0, 128, 2, 16, 16, False, 0),
          (64, 0, 128, 1, 18, 34, False, 3), (64, 0, 128, 1, 18, 34, False, 0), (128, 0, 64, 1, 16, 16, False, 0)]:
    case(*c)
