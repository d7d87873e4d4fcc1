"""fp32 1-D Winograd F(2,3) 3x3 convolution (selunet_conv3x3_wino, conv3x3_wino_persist_kernel)
against torch's conv2d / conv2d input gradient in fp64 on the CPU: forward with the BN-statistics
epilogue and torch.cat sources with folded BN+ReLU staging, data gradient with the split (ConvTranspose
bias column sums) and BN-backward-sums epilogues, and the Winograd weight pack.

Tolerance: 2e-6 of the tensor's max magnitude against the fp64 result (the direct fp32 kernel lands
at ~3e-7 on these shapes, the Winograd form at ~2x that: measured 1D F(2,3) relative RMS error
3.1e-7 vs 1.8e-7 direct at C = 512)."""
import pytest
import torch
import torch.nn.functional as F

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from tests.test_gpu_kernels import bn_fold, check_bnb_sums, gen, halo_wgs, nchw, nhwc, rel  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 2e-6


def pack_wino(w, dgrad=True):
    """Winograd operands of a conv3x3 weight [co][ci][3][3] through selunet_pack_weights."""
    co, ci = w.shape[:2]
    wd = w.to(DEV).contiguous()
    fwd = torch.empty(co, 12 * ci, device=DEV)
    dg = torch.empty(ci, 12 * co, device=DEV) if dgrad else None
    pl = K.PackList()
    pl.d[0] = K.PackDesc(K.ptr(wd), K.ptr(fwd), K.ptr(dg), K.PACK_CONV3X3_WINO, co, ci, 12 * ci, 0)
    pl.n = 1
    K.call("selunet_pack_weights", pl, K.F32, K.stream_ptr())
    return fwd, dg


def wino_u(w):
    """[co][12*ci] reference Winograd weights: k = (dy*4 + xi)*ci + c."""
    w = w.double()
    g0, g1, g2 = w[..., 0], w[..., 1], w[..., 2]  # [co][ci][dy]
    u = torch.stack([g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2], 3)  # [co][ci][dy][xi]
    return u.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def test_wino_pack():
    w = gen(64, 96, 3, 3, seed=1, scale=0.1)
    fwd, dg = pack_wino(w)
    torch.cuda.synchronize()
    assert rel(fwd, wino_u(w)) < 1e-7
    wt = w.flip(2, 3).transpose(0, 1)  # the data-gradient conv's kernel
    assert rel(dg, wino_u(wt)) < 1e-7


def test_wino_eligibility():
    ok = lambda *a: K.query("selunet_conv3x3_wino_ok", *a)  # noqa: E731
    assert ok(32, 32, 64, 64, 64) == 1
    assert ok(32, 32, 32, 32, 64) == 0    # one channel chunk: the weights-resident kernel
    assert ok(8, 8, 64, 64, 64) == 0      # below the 16x16 halo tile
    assert ok(32, 30, 64, 64, 64) == 1
    assert ok(32, 31, 64, 64, 64) == 0    # odd width: an output pair would straddle the edge
    assert ok(32, 32, 64, 64, 96) == 0


@pytest.mark.parametrize("cin0,cin1,cout,n,h,w,xform", [
    (64, 0, 64, 2, 16, 16, True),
    (64, 64, 128, 1, 16, 48, True),     # two sources (torch.cat), BN = 128
    (128, 0, 256, 2, 20, 24, True),     # partial edge tiles
    (256, 0, 128, 2, 32, 32, False),
    (128, 128, 64, 1, 32, 16, True),    # two sources, BN = 64
    (64, 0, 128, 1, 18, 34, True),      # partial tiles in both directions, even width
])
@pytest.mark.parametrize("wgs", [0, 3])
def test_wino_fwd_stats(cin0, cin1, cout, n, h, w, xform, wgs, halo_wgs):
    halo_wgs(wgs)
    x0 = gen(n, cin0, h, w, seed=1)
    x1 = gen(n, cin1, h, w, seed=2) if cin1 else None
    wt = gen(cout, cin0 + cin1, 3, 3, seed=3, scale=0.05)
    s0, t0 = bn_fold(cin0, 10)
    a = torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)) if xform else x0
    if cin1:
        s1, t1 = bn_fold(cin1, 12)
        a = torch.cat((a, torch.relu(x1 * s1.view(1, -1, 1, 1) + t1.view(1, -1, 1, 1))), 1)
    ref = F.conv2d(a.double(), wt.double(), padding=1)
    assert K.query("selunet_conv3x3_wino_ok", h, w, cin0 + cin1, cin0, cout) == 1
    u, _ = pack_wino(wt, dgrad=False)
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    keep = [d(nhwc(x0)), d(s0), d(t0)]  # K.source holds raw pointers: the tensors must stay alive
    srcs = [K.source(keep[0], cin0, keep[1] if xform else None, keep[2] if xform else None)]
    if cin1:
        keep += [d(nhwc(x1)), d(s1), d(t1)]
        srcs.append(K.source(keep[3], cin1, keep[4], keep[5]))
    M = n * h * w
    y = torch.empty(M, cout, device=DEV)
    g = K.gather(n, h, w, 9, *srcs)
    rows = K.query("selunet_gemm_stats_rows", g, cout, K.F32)
    stats = torch.empty(rows, 2, cout, device=DEV)
    ep = K.Epilogue(K.ptr(y), None, None, K.ptr(stats), K.EP_PLAIN, 0)
    K.call("selunet_conv3x3_wino", g, K.ptr(u), cout, ep, K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(nchw(y.cpu(), n, h, w), ref) < TOL
    st = stats.cpu().double().sum(0)
    r = ref.permute(1, 0, 2, 3).reshape(cout, -1)
    assert rel(st[0], r.sum(1)) < TOL and rel(st[1], (r * r).sum(1)) < TOL


@pytest.mark.parametrize("cin,cout,split,h,w", [(64, 64, 0, 32, 32), (128, 64, 64, 32, 32),
                                                (256, 128, 128, 16, 48), (128, 256, 0, 20, 24),
                                                (512, 256, 256, 16, 16)])
@pytest.mark.parametrize("wgs", [0, 3])
def test_wino_dgrad(cin, cout, split, h, w, wgs, halo_wgs):
    halo_wgs(wgs)
    n = 2
    wt = gen(cout, cin, 3, 3, seed=6, scale=0.05)
    dy = gen(n, cout, h, w, seed=7)
    x = gen(n, cin, h, w, seed=8).double().requires_grad_()
    (ref,) = torch.autograd.grad(F.conv2d(x, wt.double(), padding=1), x, dy.double())
    _, dg = pack_wino(wt)
    M = n * h * w
    dyd = nhwc(dy).to(DEV)  # kept alive: K.source holds the raw pointer
    g = K.gather(n, h, w, 9, K.source(dyd, cout))
    rows = K.query("selunet_gemm_stats_rows", g, cin, K.F32)
    if split:
        d0 = torch.empty(M, split, device=DEV)
        d1 = torch.empty(M, cin - split, device=DEV)
        colsum = torch.empty(rows, split, device=DEV)
        ep = K.Epilogue(K.ptr(d0), K.ptr(d1), None, None, K.EP_SPLIT, split, K.ptr(colsum))
        K.call("selunet_conv3x3_wino", g, K.ptr(dg), cin, ep, K.stream_ptr())
        got = torch.cat((nchw(d0.cpu(), n, h, w), nchw(d1.cpu(), n, h, w)), 1)
        assert rel(colsum.double().sum(0).cpu(), d0.double().sum(0).cpu()) < 1e-6
    else:
        dx = torch.empty(M, cin, device=DEV)
        yprev = gen(M, cin, seed=42).to(DEV)
        sc, sh = (gen(cin, seed=43).abs() + 0.5).to(DEV), (gen(cin, seed=44) * 0.3).to(DEV)
        mean, invstd = (gen(cin, seed=45) * 0.1).to(DEV), (gen(cin, seed=46).abs() + 0.5).to(DEV)
        slab = torch.empty(rows, 3, cin, device=DEV)
        ep = K.Epilogue(K.ptr(dx), None, None, None, K.EP_PLAIN, 0)
        ep.bnb = K.BnBwdStats(K.ptr(yprev), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
        K.call("selunet_conv3x3_wino", g, K.ptr(dg), cin, ep, K.stream_ptr())
        got = nchw(dx.cpu(), n, h, w)
        check_bnb_sums(slab, dx, yprev, sc, sh, mean, invstd)
    torch.cuda.synchronize()
    assert rel(got, ref) < TOL


def test_wino_rejects_ineligible():
    n, h, w, c = 1, 8, 8, 64
    x = torch.zeros(n * h * w, c, device=DEV)
    u = torch.zeros(64, 12 * c, device=DEV)
    y = torch.empty(n * h * w, 64, device=DEV)
    ep = K.Epilogue(K.ptr(y), None, None, None, K.EP_PLAIN, 0)
    with pytest.raises(K.SelunetError):
        K.call("selunet_conv3x3_wino", K.gather(n, h, w, 9, K.source(x, c)), K.ptr(u), 64, ep, K.stream_ptr())


@pytest.mark.parametrize("cin0,cin1,cout,xform,n,h,w", [
    (64, 0, 64, True, 2, 16, 16),
    (64, 64, 128, True, 2, 16, 16),     # two sources (torch.cat), BN+ReLU staging
    (128, 0, 256, False, 1, 20, 36),    # ragged 8x8 tiles in both directions
    (256, 0, 64, True, 3, 12, 18),      # ragged rows, odd tile counts
])
def test_wino_wgrad(cin0, cin1, cout, xform, n, h, w):
    """fp32 Winograd weight gradient (conv3x3_wgrad_wino_f32_kernel + the plane reduction) through
    selunet_gemm_wgrad_ws_to (the Conv2d weight layout) and selunet_gemm_wgrad_ws (packed), against
    torch's conv2d weight gradient in fp64; the two entry points agree bit for bit."""
    x0 = gen(n, cin0, h, w, seed=9)
    s0, t0 = bn_fold(cin0, 20)
    a = torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)) if xform else x0
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    keep = [d(nhwc(x0)), d(s0), d(t0)]
    srcs = [K.source(keep[0], cin0, keep[1] if xform else None, keep[2] if xform else None)]
    if cin1:
        x1 = gen(n, cin1, h, w, seed=10)
        s1, t1 = bn_fold(cin1, 22)
        a = torch.cat((a, torch.relu(x1 * s1.view(1, -1, 1, 1) + t1.view(1, -1, 1, 1))), 1)
        keep += [d(nhwc(x1)), d(s1), d(t1)]
        srcs.append(K.source(keep[3], cin1, keep[4], keep[5]))
    cin = cin0 + cin1
    wt = gen(cout, cin, 3, 3, seed=11, scale=0.05).double().requires_grad_()
    dy = gen(n, cout, h, w, seed=12)
    (ref,) = torch.autograd.grad(F.conv2d(a.double(), wt, padding=1), wt, dy.double())
    dyd = d(nhwc(dy))
    gp, gq = K.gather(n, h, w, 1, K.source(dyd, cout)), K.gather(n, h, w, 9, *srcs)
    assert K.query("selunet_gemm_kernel_name", gp, gq, 0, 0, K.F32).decode() == "conv3x3_wgrad_wino_f32<64>"
    wsb = K.query("selunet_gemm_wgrad_ws_bytes", gp, gq, K.F32)
    ws = torch.empty(wsb // 4, device=DEV)
    out = torch.full((cout, cin, 3, 3), float("nan"), device=DEV)
    K.call("selunet_gemm_wgrad_ws_to", gp, gq, None, K.ptr(ws), wsb, K.WG_CONV3X3, K.ptr(out), K.F32, K.stream_ptr())
    ld = K.query("selunet_wgrad_ld", 9 * cin)
    packed = torch.full((cout, ld), float("nan"), device=DEV)
    K.call("selunet_gemm_wgrad_ws", gp, gq, K.ptr(packed), K.ptr(ws), wsb, K.F32, K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(out.cpu(), ref) < TOL
    unpacked = packed[:, :9 * cin].reshape(cout, 9, cin).permute(0, 2, 1).reshape(cout, cin, 3, 3)
    assert torch.equal(unpacked, out) and torch.all(packed[:, 9 * cin:] == 0)
