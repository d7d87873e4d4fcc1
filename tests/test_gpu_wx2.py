"""fp32 3x3 convolution on split-fp16 operands as a 1-D Winograd F(2,3) (selunet_conv3x3_wx2,
conv3x3_wx2_kernel) against torch's conv2d / conv2d input gradient in fp64 on the CPU: the weight pack
(SELUNET_PACK_CONV3X3_WX2: U values, planes in the order 0, 2, 1, 3), the forward with the BN-statistics
epilogue and torch.cat sources with folded BN+ReLU staging, ragged edge tiles, the data gradient with
the split (ConvTranspose bias column sums) and BN-backward-sums epilogues, and persistent workgroups
over several tiles.

Tolerance: 2e-6 of the tensor's max magnitude against the fp64 result, as the exact fp32 Winograd
kernel (tests/test_gpu_wino.py) and the direct split-fp16 kernel (tests/test_gpu_x2.py): V and U are
formed in fp32 / fp64 and then carry 22 significant bits each; the transform adds one fp32 rounding
(measured: relative RMS 3.1e-7 for the fp32 Winograd form vs 1.8e-7 direct at C = 512)."""
import pytest
import torch
import torch.nn.functional as F

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from tests.test_gpu_kernels import bn_fold, check_bnb_sums, gen, halo_wgs, nchw, nhwc, rel  # noqa: F401
from tests.test_gpu_x2 import word

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 2e-6


@pytest.fixture(autouse=True)
def wx2_on():
    """selunet_conv3x3_wx2_ok admits layers only with SELUNET_OPT_WX2 set (off by default: measured slower
    than the direct split-fp16 kernel); the kernel itself is tested here either way."""
    prev = K.set_option("WX2", 1)
    yield
    K.set_option("WX2", prev)


def pack_wx2(w, dgrad=True):
    co, ci = w.shape[:2]
    wd = w.to(DEV).contiguous()
    fwd = torch.empty(co * 12 * ci + co, device=DEV)
    dg = torch.empty(ci * 12 * co + ci, device=DEV) if dgrad else None
    pl = K.PackList()
    pl.d[0] = K.PackDesc(K.ptr(wd), K.ptr(fwd), K.ptr(dg), K.PACK_CONV3X3_WX2, co, ci, 12 * ci, 0)
    pl.n = 1
    K.call("selunet_pack_weights", pl, K.F32, K.stream_ptr())
    return fwd, dg


def unpack_wx2(buf, rows, kch):
    """fp64 U[rows][dy][xi][kch] a Winograd split-fp16 pack holds: blocks (k / 16, dy, q) of 16 h + 16 l."""
    m = buf[: rows * 12 * kch].cpu().view(torch.float16).reshape(rows, kch // 16, 3, 4, 2, 16).double()
    v = (m[..., 0, :] + m[..., 1, :]) * buf[rows * 12 * kch:].cpu().double().view(rows, 1, 1, 1, 1)
    v = v[:, :, :, [0, 2, 1, 3]]  # stored planes q = 0, 2, 1, 3 -> xi
    return v.permute(0, 2, 3, 1, 4).reshape(rows, 3, 4, kch)


def u_ref(k):
    """Winograd U of kernel rows k[..., 3] -> [..., 4]."""
    g0, g1, g2 = k[..., 0], k[..., 1], k[..., 2]
    return torch.stack((g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2), -1)


def test_wx2_pack():
    w = gen(64, 96, 3, 3, seed=1, scale=0.1)
    w[5] *= 1e-3  # rows of very different ranges: one scale per row
    fwd, dg = pack_wx2(w)
    torch.cuda.synchronize()
    ref = u_ref(w.double()).permute(0, 2, 3, 1)  # [co][dy][xi][ci]
    got = unpack_wx2(fwd, 64, 96)
    tol = ref.abs().amax((1, 2, 3), keepdim=True) * 2.0 ** -20
    assert ((got - ref).abs() <= tol).all()
    wt = w.flip(2, 3).transpose(0, 1)  # the data-gradient conv's kernel [ci][co][3][3]
    ref_d = u_ref(wt.double()).permute(0, 2, 3, 1)
    got_d = unpack_wx2(dg, 96, 64)
    tol_d = ref_d.abs().amax((1, 2, 3), keepdim=True) * 2.0 ** -20
    assert ((got_d - ref_d).abs() <= tol_d).all()


def test_wx2_eligibility():
    ok = lambda *a: K.query("selunet_conv3x3_wx2_ok", *a)  # noqa: E731
    assert ok(32, 32, 64, 64, 128) == 1
    assert ok(32, 32, 64, 64, 64) == 1     # 64-column tiles
    assert ok(32, 32, 64, 64, 96) == 0
    assert ok(32, 32, 32, 32, 128) == 0    # one direct-kernel chunk
    assert ok(8, 8, 64, 64, 128) == 0      # below the 16x16 tile
    assert ok(32, 31, 64, 64, 128) == 0    # output pairs need an even width
    assert ok(32, 34, 128, 64, 256) == 1


@pytest.mark.parametrize("cin0,cin1,cout,n,h,w,xform", [
    (64, 0, 128, 2, 16, 16, True),
    (64, 64, 128, 1, 16, 48, True),     # two sources (torch.cat)
    (128, 0, 256, 2, 20, 24, True),     # partial edge tiles
    (256, 0, 128, 2, 32, 32, False),
    (128, 128, 256, 1, 32, 16, True),   # two sources, two column tiles
    (64, 0, 128, 1, 18, 34, True),      # partial tiles in both directions
    (64, 0, 64, 2, 32, 32, True),       # BN = 64
    (64, 64, 64, 1, 20, 48, True),      # BN = 64, two sources, partial tiles
])
@pytest.mark.parametrize("wgs", [0, 3])
def test_wx2_fwd_stats(cin0, cin1, cout, n, h, w, xform, wgs, halo_wgs):
    halo_wgs(wgs)
    x0 = gen(n, cin0, h, w, seed=1)
    x1 = gen(n, cin1, h, w, seed=2) * 1e-3 if cin1 else None  # sources of different ranges
    wt = gen(cout, cin0 + cin1, 3, 3, seed=3, scale=0.05)
    s0, t0 = bn_fold(cin0, 10)
    a0 = torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)) if xform else x0
    a = a0
    if cin1:
        s1, t1 = bn_fold(cin1, 12)
        a1 = torch.relu(x1 * s1.view(1, -1, 1, 1) + t1.view(1, -1, 1, 1))
        a = torch.cat((a0, a1), 1)
    ref = F.conv2d(a.double(), wt.double(), padding=1)
    assert K.query("selunet_conv3x3_wx2_ok", h, w, cin0 + cin1, cin0, cout) == 1
    u, _ = pack_wx2(wt, dgrad=False)
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    keep = [d(nhwc(x0)), d(s0), d(t0)]  # K.source holds raw pointers: the tensors must stay alive
    srcs = [K.source(keep[0], cin0, keep[1] if xform else None, keep[2] if xform else None)]
    am0, am1 = word(a0.abs().max() * 1.5), None
    if cin1:
        keep += [d(nhwc(x1)), d(s1), d(t1)]
        srcs.append(K.source(keep[3], cin1, keep[4], keep[5]))
        am1 = word(a1.abs().max())
    M = n * h * w
    y = torch.empty(M, cout, device=DEV)
    g = K.gather(n, h, w, 9, *srcs)
    rows = K.query("selunet_conv3x3_x2_stats_rows", g, cout)
    stats = torch.empty(rows, 2, cout, device=DEV)
    amo = torch.zeros(1, device=DEV)
    ep = K.Epilogue(K.ptr(y), None, None, K.ptr(stats), K.EP_PLAIN, 0)
    ep.amax = K.ptr(amo)
    K.call("selunet_conv3x3_wx2", g, K.ptr(u), cout, ep, K.ptr(am0), K.ptr(am1), K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(nchw(y.cpu(), n, h, w), ref) < TOL
    st = stats.cpu().double().sum(0)
    r = ref.permute(1, 0, 2, 3).reshape(cout, -1)
    assert rel(st[0], r.sum(1)) < TOL and rel(st[1], (r * r).sum(1)) < TOL
    assert amo.item() == y.abs().max().item()


@pytest.mark.parametrize("cin,cout,split,h,w", [(128, 64, 0, 32, 32), (128, 128, 64, 32, 32),
                                                (256, 128, 128, 16, 48), (128, 256, 0, 20, 24),
                                                (512, 256, 256, 16, 16), (256, 512, 0, 32, 32),
                                                (64, 64, 0, 32, 32), (64, 128, 0, 24, 16)])
@pytest.mark.parametrize("wgs", [0, 3])
def test_wx2_dgrad(cin, cout, split, h, w, wgs, halo_wgs):
    """Gradient-sized operands (1e-9 scale): the range word rescales them into the fp16 range. The data
    gradient's output has cin columns (the weight pack's dgrad half)."""
    halo_wgs(wgs)
    n = 2
    wt = gen(cout, cin, 3, 3, seed=6, scale=0.05)
    dy = gen(n, cout, h, w, seed=7) * 1e-9
    x = gen(n, cin, h, w, seed=8).double().requires_grad_()
    (ref,) = torch.autograd.grad(F.conv2d(x, wt.double(), padding=1), x, dy.double())
    assert K.query("selunet_conv3x3_wx2_ok", h, w, cout, cout, cin) == 1
    _, dg = pack_wx2(wt)
    M = n * h * w
    dyd = nhwc(dy).to(DEV)  # kept alive: K.source holds the raw pointer
    am = word(dy.abs().max())
    g = K.gather(n, h, w, 9, K.source(dyd, cout))
    rows = K.query("selunet_conv3x3_x2_stats_rows", g, cin)
    if split:
        d0 = torch.empty(M, split, device=DEV)
        d1 = torch.empty(M, cin - split, device=DEV)
        colsum = torch.empty(rows, split, device=DEV)
        ep = K.Epilogue(K.ptr(d0), K.ptr(d1), None, None, K.EP_SPLIT, split, K.ptr(colsum))
        K.call("selunet_conv3x3_wx2", g, K.ptr(dg), cin, ep, K.ptr(am), None, K.stream_ptr())
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
        K.call("selunet_conv3x3_wx2", g, K.ptr(dg), cin, ep, K.ptr(am), None, K.stream_ptr())
        got = nchw(dx.cpu(), n, h, w)
        check_bnb_sums(slab, dx, yprev, sc, sh, mean, invstd)
    torch.cuda.synchronize()
    assert rel(got, ref) < TOL


def test_wx2_matches_direct_x2_statistics_rows():
    """Same statistics slab rows as the direct split-fp16 kernel (the engine sizes slabs by the query)."""
    x = torch.zeros(2 * 64 * 64, 128, device=DEV)
    g = K.gather(2, 64, 64, 9, K.source(x, 128))
    assert K.query("selunet_conv3x3_x2_stats_rows", g, 256) == K.query("selunet_gemm_stats_rows", g, 256, K.F32)
