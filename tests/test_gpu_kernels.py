"""Per-kernel parity of libselunet.so against plain PyTorch fp32 on the CPU (the oracle's ops).

Called through the C-ABI (ctypes) exactly as the product path calls it. fp32 tolerance:
1e-4 relative to the tensor's max magnitude; exact fp32 MFMA accumulation differs from
oneDNN's summation order only in rounding.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))


def nhwc(t):  # [N,C,H,W] -> [N*H*W, C]
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).contiguous()


def nchw(t, n, h, w):
    return t.reshape(n, h, w, -1).permute(0, 3, 1, 2)


@pytest.fixture
def halo_wgs():
    """Set the persistent halo kernel's workgroup target for one test (0 = default), restored after."""
    prev = []

    def set_(wgs):
        prev.append(K.query("selunet_set_halo_workgroups", wgs))

    yield set_
    if prev:
        K.query("selunet_set_halo_workgroups", prev[0])


@pytest.fixture
def gather_wgs():
    """Set the persistent gather GEMM's workgroup target for one test (-1 = default, 0 = one tile per
    workgroup), restored after."""
    prev = []

    def set_(wgs):
        prev.append(K.query("selunet_set_gather_workgroups", wgs))

    yield set_
    if prev:
        K.query("selunet_set_gather_workgroups", prev[0])


@pytest.fixture
def kernel_option():
    """Set library options (selunet_set_option) for one test, restored after."""
    prev = []

    def set_(variant):
        if variant is not None:
            prev.append((variant[0], K.set_option(*variant)))

    yield set_
    for name, v in reversed(prev):
        K.set_option(name, v)


# kernel-selection alternatives the bf16 persistent-kernel tests also run under (the 16x16x32 MFMA form and
# single-chunk layers on the persistent kernel were retired in round 6 after losing every A/B)
BF16_VARIANTS = [None]


def gen(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def bn_fold(c, seed):
    scale = gen(c, seed=seed).abs() + 0.5
    shift = gen(c, seed=seed + 1) * 0.3
    return scale, shift


def pack(w, dt=torch.float32):
    co, ci = w.shape[:2]
    bke = 128 // torch.empty((), dtype=dt).element_size()
    kpad = (9 * ci + bke - 1) // bke * bke
    fwd = torch.empty(co, kpad, dtype=dt, device=DEV)
    dg = torch.empty(ci, 9 * co, dtype=dt, device=DEV)
    wd = w.to(DEV).contiguous()
    K.call("selunet_pack_conv3x3", K.ptr(wd), co, ci, kpad, K.ptr(fwd), K.ptr(dg), K.dtype_code(dt), K.stream_ptr())
    return fwd, dg, kpad


@pytest.mark.parametrize("cin0,cin1,cout,n,h,w,xform", [
    (64, 0, 64, 2, 16, 16, True),
    (128, 0, 256, 1, 8, 12, False),
    (64, 64, 128, 2, 8, 8, True),      # two-source (torch.cat) gather
    (256, 256, 256, 1, 4, 4, True),
    (64, 0, 128, 3, 5, 7, True),       # M not a multiple of the 128-row tile
    (64, 0, 64, 2, 32, 32, True),      # 16x16 halo-tile kernel
    (64, 64, 128, 1, 16, 48, True),    # halo kernel, two sources, BN = 128
    (128, 0, 256, 2, 20, 24, True),    # halo kernel, partial edge tiles
    (32, 0, 64, 2, 24, 20, True),      # one fp32 channel chunk: weights-resident persistent kernel
])
@pytest.mark.parametrize("wgs", [0, 3])
def test_conv3x3_fwd_stats(cin0, cin1, cout, n, h, w, xform, wgs, halo_wgs):
    """wgs = 3: the persistent multi-chunk halo kernel with 3 workgroup rows, so every workgroup
    walks several (unevenly many) tiles and accumulates its statistics over them."""
    halo_wgs(wgs)
    x0 = gen(n, cin0, h, w, seed=1)
    x1 = gen(n, cin1, h, w, seed=2) if cin1 else None
    wt = gen(cout, cin0 + cin1, 3, 3, seed=3, scale=0.05)
    s0, t0 = bn_fold(cin0, 10)
    s1, t1 = bn_fold(cin1, 12) if cin1 else (None, None)
    # reference: transform (BN fold + relu) applied to source 1 only when it is a "skip" source
    a0 = torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)) if xform else x0
    a = a0
    if cin1:
        a1 = torch.relu(x1 * s1.view(1, -1, 1, 1) + t1.view(1, -1, 1, 1))
        a = torch.cat((a0, a1), 1)
    ref = F.conv2d(a, wt, padding=1)
    fwd, _, kpad = pack(wt)
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    x0d, s0d, t0d = d(nhwc(x0)), d(s0), d(t0)
    srcs = [K.source(x0d, cin0, s0d if xform else None, t0d if xform else None)]
    if cin1:
        x1d, s1d, t1d = d(nhwc(x1)), d(s1), d(t1)
        srcs.append(K.source(x1d, cin1, s1d, t1d))
    M = n * h * w
    y = torch.empty(M, cout, device=DEV)
    g = K.gather(n, h, w, 9, *srcs)
    rows = K.query("selunet_gemm_stats_rows", g, cout, K.F32)
    stats = torch.empty(rows, 2, cout, device=DEV)
    ep = K.Epilogue(K.ptr(y), None, None, K.ptr(stats), K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", g, K.ptr(fwd), cout, kpad, ep, K.F32, K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(nchw(y.cpu(), n, h, w), ref) < TOL
    st = stats.cpu().double().sum(0)
    r = ref.double().permute(1, 0, 2, 3).reshape(cout, -1)
    assert rel(st[0], r.sum(1)) < TOL and rel(st[1], (r * r).sum(1)) < TOL


def test_conv3x3_fwd_small_c_nchw():
    n, h, w = 2, 16, 16
    x = gen(n, 3, h, w, seed=4)
    wt = gen(64, 3, 3, 3, seed=5, scale=0.2)
    ref = F.conv2d(x, wt, padding=1)
    fwd, _, kpad = pack(wt)
    xd = x.to(DEV).contiguous()
    y = torch.empty(n * h * w, 64, device=DEV)
    ep = K.Epilogue(K.ptr(y), None, None, None, K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", K.gather(n, h, w, 9, K.source(xd, 3, layout=1)), K.ptr(fwd), 64, kpad, ep, K.F32,
           K.stream_ptr())
    assert rel(nchw(y.cpu(), n, h, w), ref) < TOL


@pytest.mark.parametrize("cin,cout,split,h,w", [(64, 64, 0, 8, 8), (128, 64, 64, 8, 8), (512, 256, 256, 8, 8),
                                                (64, 128, 0, 8, 8), (64, 64, 0, 32, 32), (128, 64, 64, 32, 32),
                                                (256, 128, 128, 16, 48), (64, 32, 0, 24, 20), (128, 32, 64, 16, 40)])
@pytest.mark.parametrize("wgs", [0, 3])
def test_conv3x3_dgrad(cin, cout, split, h, w, wgs, halo_wgs, gather_wgs):
    """wgs = 3 also sets the generic gather GEMM (the 8x8 cases, 3 row tiles at n = 6) to one workgroup
    row: one workgroup walks every tile and accumulates the column / BN-backward sums over them."""
    halo_wgs(wgs)
    gather_wgs(wgs - 2 if wgs else -1)
    n = 6 if h == 8 else 2
    wt = gen(cout, cin, 3, 3, seed=6, scale=0.05)
    dy = gen(n, cout, h, w, seed=7)
    x = gen(n, cin, h, w, seed=8).requires_grad_()
    y = F.conv2d(x, wt, padding=1)
    (ref,) = torch.autograd.grad(y, x, dy)
    _, dg, _ = pack(wt)
    dyd = nhwc(dy).to(DEV)
    M = n * h * w
    g = K.gather(n, h, w, 9, K.source(dyd, cout))
    rows = K.query("selunet_gemm_stats_rows", g, cin, K.F32)
    if split:
        d0 = torch.empty(M, split, device=DEV)
        d1 = torch.empty(M, cin - split, device=DEV)
        colsum = torch.empty(rows, split, device=DEV)
        ep = K.Epilogue(K.ptr(d0), K.ptr(d1), None, None, K.EP_SPLIT, split, K.ptr(colsum))
        K.call("selunet_gemm_gather", g, K.ptr(dg), cin, 9 * cout, ep, K.F32, K.stream_ptr())
        got = torch.cat((nchw(d0.cpu(), n, h, w), nchw(d1.cpu(), n, h, w)), 1)
        # column sums of the up-sampled half (the ConvTranspose2d bias gradient)
        assert rel(colsum.double().sum(0).cpu(), d0.double().sum(0).cpu()) < 1e-6
    else:
        dx = torch.empty(M, cin, device=DEV)
        # with the fused BatchNorm-backward sums of the producing layer (y, folded BN, batch stats)
        yprev = gen(M, cin, seed=42).to(DEV)
        sc, sh = (gen(cin, seed=43).abs() + 0.5).to(DEV), (gen(cin, seed=44) * 0.3).to(DEV)
        mean, invstd = (gen(cin, seed=45) * 0.1).to(DEV), (gen(cin, seed=46).abs() + 0.5).to(DEV)
        slab = torch.empty(rows, 3, cin, device=DEV)
        ep = K.Epilogue(K.ptr(dx), None, None, None, K.EP_PLAIN, 0)
        ep.bnb = K.BnBwdStats(K.ptr(yprev), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
        K.call("selunet_gemm_gather", g, K.ptr(dg), cin, 9 * cout, ep, K.F32, K.stream_ptr())
        got = nchw(dx.cpu(), n, h, w)
        check_bnb_sums(slab, dx, yprev, sc, sh, mean, invstd)
    assert rel(got, ref) < TOL


@pytest.mark.parametrize("cin0,cin1,cout,xform,small,h,w", [
    (64, 0, 64, True, False, 16, 16), (64, 64, 128, True, False, 16, 16), (128, 0, 256, False, False, 16, 16),
    (3, 0, 64, False, True, 16, 16),
    (64, 0, 64, True, False, 20, 36),     # fp32 halo wgrad: ragged 8x8 tiles, tap groups (BI = 64)
    (128, 64, 128, True, False, 12, 16),  # fp32 halo wgrad: BI = 128, two sources, ragged rows
    (64, 0, 128, False, False, 8, 8),     # generic fp32 wgrad (width below the halo tile)
])
def test_conv3x3_wgrad(cin0, cin1, cout, xform, small, h, w):
    """fp32 weight gradient through both entry points: selunet_gemm_wgrad (fp32 atomics) and the
    deterministic split-partials path selunet_gemm_wgrad_ws (fixed-order reduction)."""
    n = 2
    x0 = gen(n, cin0, h, w, seed=9)
    x1 = gen(n, cin1, h, w, seed=10) if cin1 else None
    s0, t0 = bn_fold(cin0, 20)
    s1, t1 = bn_fold(cin1, 22) if cin1 else (None, None)
    a = torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)) if xform else x0
    if cin1:
        a = torch.cat((a, torch.relu(x1 * s1.view(1, -1, 1, 1) + t1.view(1, -1, 1, 1))), 1)
    cin = cin0 + cin1
    wt = gen(cout, cin, 3, 3, seed=11, scale=0.05).requires_grad_()
    dy = gen(n, cout, h, w, seed=12)
    y = F.conv2d(a, wt, padding=1)
    (ref,) = torch.autograd.grad(y, wt, dy)
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    if small:
        srcs = [K.source(d(x0), cin0, layout=1)]
        keep = [d(x0)]
        srcs = [K.source(keep[0], cin0, layout=1)]
    else:
        keep = [d(nhwc(x0)), d(s0), d(t0)]
        srcs = [K.source(keep[0], cin0, keep[1] if xform else None, keep[2] if xform else None)]
        if cin1:
            keep += [d(nhwc(x1)), d(s1), d(t1)]
            srcs.append(K.source(keep[3], cin1, keep[4], keep[5]))
    dyd = d(nhwc(dy))
    ld = K.query("selunet_wgrad_ld", 9 * cin)
    packed = torch.zeros(cout, ld, device=DEV)
    K.call("selunet_gemm_wgrad", K.gather(n, h, w, 1, K.source(dyd, cout)), K.gather(n, h, w, 9, *srcs),
           K.ptr(packed), K.F32, K.stream_ptr())
    out = torch.empty(cout, cin, 3, 3, device=DEV)
    K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), cout, cin, ld, K.ptr(out), K.stream_ptr())
    assert rel(out.cpu(), ref) < TOL
    if not small:
        gp, gq = K.gather(n, h, w, 1, K.source(dyd, cout)), K.gather(n, h, w, 9, *srcs)
        det = wgrad_ws(gp, gq, packed, dtype=K.F32)
        K.call("selunet_unpack_conv3x3_grad", K.ptr(det), cout, cin, ld, K.ptr(out), K.stream_ptr())
        assert rel(out.cpu(), ref) < TOL


@pytest.mark.parametrize("cin,cout", [(512, 256), (128, 64)])
@pytest.mark.parametrize("gwgs", [-1, 0, 3, 16])
def test_convT_fwd_bwd(cin, cout, gwgs, gather_wgs):
    """4 row tiles (the last one ragged): one tile per workgroup (0), every tile in one workgroup
    (3), two tiles per workgroup (16 at 1024 columns) and the default persistent launch."""
    gather_wgs(gwgs)
    n, h, w = 2, 13, 18
    x = gen(n, cin, h, w, seed=13)
    s, t = bn_fold(cin, 30)
    a = torch.relu(x * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1)).requires_grad_()
    wt = gen(cin, cout, 2, 2, seed=14, scale=0.05).requires_grad_()
    b = gen(cout, seed=15).requires_grad_()
    y = F.conv_transpose2d(a, wt, b, stride=2)
    dy = gen(*y.shape, seed=16)
    ga, gw, gb = torch.autograd.grad(y, (a, wt, b), dy)
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    xd, sd, td, wd, bd = d(nhwc(x)), d(s), d(t), d(wt.detach()), d(b.detach())
    fwd = torch.empty(4 * cout, cin, device=DEV)
    dg = torch.empty(cin, 4 * cout, device=DEV)
    K.call("selunet_pack_convT", K.ptr(wd), cin, cout, K.ptr(fwd), K.ptr(dg), K.F32, K.stream_ptr())
    up = torch.empty(n * 2 * h * 2 * w, cout, device=DEV)
    ep = K.Epilogue(K.ptr(up), None, K.ptr(bd), None, K.EP_SCATTER2X, 0)
    K.call("selunet_gemm_gather", K.gather(n, h, w, 1, K.source(xd, cin, sd, td)), K.ptr(fwd), 4 * cout, cin, ep,
           K.F32, K.stream_ptr())
    assert rel(nchw(up.cpu(), n, 2 * h, 2 * w), y) < TOL
    # backward
    dud = d(nhwc(dy))
    da = torch.empty(n * h * w, cin, device=DEV)
    ep = K.Epilogue(K.ptr(da), None, None, None, K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", K.gather(n, h, w, 4, K.source(dud, cout)), K.ptr(dg), cin, 4 * cout, ep, K.F32,
           K.stream_ptr())
    assert rel(nchw(da.cpu(), n, h, w), ga) < TOL
    ld = K.query("selunet_wgrad_ld", 4 * cout)
    packed = torch.zeros(cin, ld, device=DEV)
    K.call("selunet_gemm_wgrad", K.gather(n, h, w, 1, K.source(xd, cin, sd, td)),
           K.gather(n, h, w, 4, K.source(dud, cout)), K.ptr(packed), K.F32, K.stream_ptr())
    gwd = torch.empty(cin, cout, 2, 2, device=DEV)
    K.call("selunet_unpack_convT_grad", K.ptr(packed), cin, cout, K.ptr(gwd), K.stream_ptr())
    assert rel(gwd.cpu(), gw) < TOL
    det = wgrad_ws(K.gather(n, h, w, 1, K.source(xd, cin, sd, td)), K.gather(n, h, w, 4, K.source(dud, cout)), packed,
                   dtype=K.F32)  # split partials + fixed-order reduction
    K.call("selunet_unpack_convT_grad", K.ptr(det), cin, cout, K.ptr(gwd), K.stream_ptr())
    assert rel(gwd.cpu(), gw) < TOL
    Mu = n * 4 * h * w
    rows = K.query("selunet_channel_slab_rows", Mu)
    slab = torch.empty(rows, cout, device=DEV)
    K.call("selunet_channel_sum", K.ptr(dud), Mu, cout, K.ptr(slab), K.F32, K.stream_ptr())
    assert rel(slab.sum(0).cpu(), gb) < TOL


def test_maxpool_ties_and_backward():
    """Windows with exact ties (post-ReLU zeros, duplicated maxima): gradient goes to the first
    maximum in row-major window order, as ATen's max_pool2d_with_indices."""
    n, c, h, w = 2, 64, 8, 8
    y = gen(n, c, h, w, seed=17)
    y[:, :, ::2, 1::2] = y[:, :, ::2, ::2]          # tie between (0,0) and (0,1)
    y[:, :8] = -1.0                                  # all-zero windows after ReLU
    s = torch.ones(c)
    t = torch.zeros(c)
    z = torch.relu(y).requires_grad_()
    p = F.max_pool2d(z, 2)
    dp = gen(*p.shape, seed=18)
    dskip = gen(*z.shape, seed=19)
    (gz,) = torch.autograd.grad(p, z, dp)
    gz = gz + dskip
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    yd, sd, td = d(nhwc(y)), d(s), d(t)
    out = torch.empty(n * h * w // 4, c, device=DEV)
    K.call("selunet_maxpool2_fwd", K.ptr(yd), n, h, w, c, K.ptr(sd), K.ptr(td), K.ptr(out), K.F32, K.stream_ptr())
    assert torch.equal(nchw(out.cpu(), n, h // 2, w // 2), p.detach())
    dpd, dsd = d(nhwc(dp)), d(nhwc(dskip))
    dz = torch.empty_like(yd)
    K.call("selunet_maxpool2_bwd", K.ptr(yd), n, h, w, c, K.ptr(sd), K.ptr(td), K.ptr(dpd), K.ptr(dsd), K.ptr(dz),
           None, K.F32, K.stream_ptr())
    assert torch.equal(nchw(dz.cpu(), n, h, w), gz)
    # fused BatchNorm-backward sums of dz (selunet_bn_bwd_stats)
    mean, invstd = d(gen(c, seed=40) * 0.1), d(gen(c, seed=41).abs() + 0.5)
    rows = K.query("selunet_maxpool2_bwd_slab_rows", n, h, w, c)
    slab = torch.zeros(rows, 3, c, device=DEV)
    bnb = K.BnBwdStats(K.ptr(yd), K.ptr(sd), K.ptr(td), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
    K.call("selunet_maxpool2_bwd", K.ptr(yd), n, h, w, c, K.ptr(sd), K.ptr(td), K.ptr(dpd), K.ptr(dsd), K.ptr(dz),
           bnb, K.F32, K.stream_ptr())
    assert torch.equal(nchw(dz.cpu(), n, h, w), gz)
    check_bnb_sums(slab, dz, yd, sd, td, mean, invstd)


def check_bnb_sums(slab, da, y, scale, shift, mean, invstd, tol=1e-5):
    """slab [rows][3][C] against (sum da, sum da*xhat, sum xhat), da = dA*[y*scale+shift > 0]."""
    y64, da64 = y.double(), da.double()
    m = (y64 * scale.double() + shift.double() > 0).double()
    g = da64 * m
    xh = (y64 - mean.double()) * invstd.double()
    want = torch.stack([g.sum(0), (g * xh).sum(0), xh.sum(0)])
    got = slab.double().sum(0)
    scale_ = want.abs().max(dim=1, keepdim=True).values + 1.0
    assert float(((got - want).abs() / scale_).max()) < tol


def test_bn_forward_backward_against_torch():
    n, c, h, w = 4, 128, 8, 8
    M = n * h * w
    yr = gen(n, c, h, w, seed=20) * 2 + 0.5         # pre-BN conv output without bias
    bias = gen(c, seed=21) * 0.1
    gamma = gen(c, seed=22).abs() + 0.5
    beta = gen(c, seed=23) * 0.2
    rm0, rv0 = gen(c, seed=24) * 0.1, gen(c, seed=25).abs() + 0.5
    yb = (yr + bias.view(1, -1, 1, 1)).requires_grad_()
    gam = gamma.clone().requires_grad_()
    bet = beta.clone().requires_grad_()
    rm, rv = rm0.clone(), rv0.clone()
    z = torch.relu(F.batch_norm(yb, rm, rv, gam, bet, training=True, momentum=0.1, eps=1e-5))
    dz = gen(*z.shape, seed=26)
    g_y, g_gam, g_bet = torch.autograd.grad(z, (yb, gam, bet), dz)
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    yd = d(nhwc(yr))
    r = yr.double().permute(1, 0, 2, 3).reshape(c, -1)
    sums = d(torch.cat([r.sum(1), (r * r).sum(1)]))
    rmd, rvd = d(rm0), d(rv0)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    mean, invstd, scale, shift = (torch.empty(c, device=DEV) for _ in range(4))
    biasd, gammad, betad = d(bias), d(gamma), d(beta)  # keep device tensors alive across the launch
    K.call("selunet_bn_finalize", K.ptr(sums), M, c, K.ptr(biasd), K.ptr(gammad), K.ptr(betad), K.ptr(rmd),
           K.ptr(rvd), K.ptr(nbt), 0.1, 1e-5, 1, K.ptr(mean), K.ptr(invstd), K.ptr(scale), K.ptr(shift),
           K.stream_ptr())
    assert rel(rmd.cpu(), rm) < 1e-5 and rel(rvd.cpu(), rv) < 1e-5 and int(nbt) == 1
    zz = torch.relu(yd * scale + shift)
    assert rel(nchw(zz.cpu(), n, h, w), z) < TOL
    dzd = d(nhwc(dz))
    rows = K.query("selunet_channel_slab_rows", M)
    slab = torch.empty(rows, 3, c, device=DEV)
    K.call("selunet_bn_bwd_reduce", K.ptr(dzd), K.ptr(yd), M, c, K.ptr(scale), K.ptr(shift), K.ptr(mean),
           K.ptr(invstd), K.ptr(slab), K.F32, K.stream_ptr())
    s3 = slab.double().sum(0).reshape(-1).contiguous()
    dgam, dbet, dbias = (torch.empty(c, device=DEV) for _ in range(3))
    coef = torch.empty(3, c, device=DEV)
    K.call("selunet_bn_bwd_finalize", K.ptr(s3), M, c, K.ptr(gammad), K.ptr(invstd), K.ptr(dgam), K.ptr(dbet),
           K.ptr(dbias), K.ptr(coef), K.stream_ptr())
    assert rel(dgam.cpu(), g_gam) < TOL and rel(dbet.cpu(), g_bet) < TOL
    dy = torch.empty_like(yd)
    K.call("selunet_bn_bwd_apply", K.ptr(dzd), K.ptr(yd), M, c, K.ptr(scale), K.ptr(shift), K.ptr(mean),
           K.ptr(invstd), K.ptr(coef), K.ptr(dy), K.F32, K.stream_ptr())
    assert rel(nchw(dy.cpu(), n, h, w), g_y) < TOL
    assert float(dbias.abs().max()) < 1e-4 * float(g_y.abs().sum(dim=(0, 2, 3)).max() + 1)


def test_reduce_rows_deterministic():
    slab = gen(3001, 70, seed=27).to(DEV)
    ws = torch.empty(K.query("selunet_reduce_ws_bytes", 70) // 8, dtype=torch.float64, device=DEV)
    outs = []
    for _ in range(2):
        o = torch.empty(70, dtype=torch.float64, device=DEV)
        K.call("selunet_reduce_rows", K.ptr(slab), 3001, 70, K.ptr(ws), K.ptr(o), None, K.stream_ptr())
        outs.append(o.cpu())
    assert torch.equal(outs[0], outs[1])
    assert rel(outs[0], slab.double().sum(0).cpu()) < 1e-12


# ---------------------------------------------------------------- fused launches (launch-count cuts)
@pytest.mark.parametrize("rows", [1, 37, 1024, 1025, 5000])
@pytest.mark.parametrize("c", [64, 192, 512])
def test_bn_stats_finalize_matches_reduce_then_finalize(rows, c):
    """selunet_bn_stats_finalize / selunet_bn_bwd_stats_finalize (one launch at <= 1024 rows, two
    above) against selunet_reduce_rows + the separate finalize kernels: fp64 sums equal to 1e-12,
    finalized outputs to fp32 rounding; bit-reproducible across calls."""
    M = 4096
    slab2 = (gen(rows, 2, c, seed=40) + torch.tensor([0.3, 1.2]).view(1, 2, 1)).to(DEV)
    slab2[:, 1] = slab2[:, 1].abs() * 3  # sum of squares stays above mean^2 * count
    slab3 = gen(rows, 3, c, seed=41).to(DEV)
    bias, gamma, beta = gen(c, seed=42).to(DEV) * 0.1, gen(c, seed=43).abs().to(DEV) + 0.5, gen(c, seed=44).to(DEV)
    ws = torch.empty(K.query("selunet_reduce_ws_bytes", 3 * c) // 8, dtype=torch.float64, device=DEV)

    def fwd_fused():
        rm, rv = torch.full((c,), 0.1, device=DEV), torch.ones(c, device=DEV)
        nbt = torch.zeros((), dtype=torch.int64, device=DEV)
        o = [torch.empty(c, device=DEV) for _ in range(4)]
        sums = torch.empty(2 * c, dtype=torch.float64, device=DEV)
        K.call("selunet_bn_stats_finalize", K.ptr(slab2), rows, K.ptr(ws), K.ptr(sums), M, c, K.ptr(bias),
               K.ptr(gamma), K.ptr(beta), K.ptr(rm), K.ptr(rv), K.ptr(nbt), 0.1, 1e-5, *[K.ptr(t) for t in o],
               K.stream_ptr())
        return sums, [rm, rv] + o, int(nbt)

    def fwd_ref():
        rm, rv = torch.full((c,), 0.1, device=DEV), torch.ones(c, device=DEV)
        nbt = torch.zeros((), dtype=torch.int64, device=DEV)
        o = [torch.empty(c, device=DEV) for _ in range(4)]
        sums = torch.empty(2 * c, dtype=torch.float64, device=DEV)
        K.call("selunet_reduce_rows", K.ptr(slab2), rows, 2 * c, K.ptr(ws), K.ptr(sums), None, K.stream_ptr())
        K.call("selunet_bn_finalize", K.ptr(sums), M, c, K.ptr(bias), K.ptr(gamma), K.ptr(beta), K.ptr(rm),
               K.ptr(rv), K.ptr(nbt), 0.1, 1e-5, 1, *[K.ptr(t) for t in o], K.stream_ptr())
        return sums, [rm, rv] + o, int(nbt)

    s_f, o_f, n_f = fwd_fused()
    s_f2, o_f2, _ = fwd_fused()
    s_r, o_r, n_r = fwd_ref()
    assert n_f == n_r == 1
    assert rel(s_f, slab2.double().sum(0).reshape(-1)) < 1e-12
    assert rel(s_f, s_r) < 1e-12
    assert torch.equal(s_f, s_f2) and all(torch.equal(a, b) for a, b in zip(o_f, o_f2))
    for a, b in zip(o_f, o_r):
        assert rel(a, b) < 1e-6

    def bwd(fused):
        sums = torch.empty(3 * c, dtype=torch.float64, device=DEV)
        invstd = o_r[3]
        o = [torch.empty(c, device=DEV) for _ in range(3)] + [torch.empty(3, c, device=DEV)]
        if fused:
            K.call("selunet_bn_bwd_stats_finalize", K.ptr(slab3), rows, K.ptr(ws), K.ptr(sums), M, c, K.ptr(gamma),
                   K.ptr(invstd), *[K.ptr(t) for t in o], K.stream_ptr())
        else:
            K.call("selunet_reduce_rows", K.ptr(slab3), rows, 3 * c, K.ptr(ws), K.ptr(sums), None, K.stream_ptr())
            K.call("selunet_bn_bwd_finalize", K.ptr(sums), M, c, K.ptr(gamma), K.ptr(invstd), *[K.ptr(t) for t in o],
                   K.stream_ptr())
        return sums, o

    s_f, o_f = bwd(True)
    s_r, o_r2 = bwd(False)
    assert rel(s_f, slab3.double().sum(0).reshape(-1)) < 1e-12 and rel(s_f, s_r) < 1e-12
    for a, b in zip(o_f[:2] + o_f[3:], o_r2[:2] + o_r2[3:]):
        assert rel(a, b) < 1e-6
    # dbias is analytically zero: only rounding noise, bounded by the terms it cancels
    assert float((o_f[2] - o_r2[2]).abs().max()) < 1e-6 * float(o_r2[0].abs().max() * M + 1)


def test_pack_weights_matches_per_tensor_packs():
    """One selunet_pack_weights launch over conv3x3 (with/without dgrad) and ConvTranspose2d
    entries equals the per-tensor pack entry points bit for bit (bf16 and fp32)."""
    specs = [("c", 64, 3, 32), ("c", 128, 64, 576), ("c", 256, 512, 4608), ("t", 256, 512, 0), ("c", 64, 128, 1152),
             ("t", 64, 128, 0)]
    for dt, code in ((torch.bfloat16, K.BF16), (torch.float32, K.F32)):
        pl = K.PackList()
        outs = []
        for i, (kind, co, ci, kpad) in enumerate(specs):
            if kind == "c":
                w = gen(co, ci, 3, 3, seed=50 + i).to(DEV)
                fwd = torch.empty(co, kpad, dtype=dt, device=DEV)
                dg = torch.empty(ci, 9 * co, dtype=dt, device=DEV) if ci != 3 else None
                ref_f, ref_d = torch.empty_like(fwd), (torch.empty_like(dg) if dg is not None else None)
                K.call("selunet_pack_conv3x3", K.ptr(w), co, ci, kpad, K.ptr(ref_f), K.ptr(ref_d), code, K.stream_ptr())
                pl.d[pl.n] = K.PackDesc(K.ptr(w), K.ptr(fwd), K.ptr(dg), K.PACK_CONV3X3, co, ci, kpad, 0)
            else:
                w = gen(ci, co, 2, 2, seed=50 + i).to(DEV)
                fwd = torch.empty(4 * co, ci, dtype=dt, device=DEV)
                dg = torch.empty(ci, 4 * co, dtype=dt, device=DEV)
                ref_f, ref_d = torch.empty_like(fwd), torch.empty_like(dg)
                K.call("selunet_pack_convT", K.ptr(w), ci, co, K.ptr(ref_f), K.ptr(ref_d), code, K.stream_ptr())
                pl.d[pl.n] = K.PackDesc(K.ptr(w), K.ptr(fwd), K.ptr(dg), K.PACK_CONVT, co, ci, 0, 0)
            pl.n += 1
            outs.append((w, fwd, dg, ref_f, ref_d))
        K.call("selunet_pack_weights", pl, code, K.stream_ptr())
        torch.cuda.synchronize()
        for w, fwd, dg, ref_f, ref_d in outs:
            assert torch.equal(fwd, ref_f)
            if dg is not None:
                assert torch.equal(dg, ref_d)


@pytest.mark.parametrize("kind,n,h,w,cp,cq", [("c", 2, 16, 16, 64, 64), ("c", 2, 32, 32, 128, 64),
                                              ("c", 1, 8, 8, 256, 512), ("t", 2, 16, 16, 128, 64),
                                              ("t", 2, 8, 8, 512, 256)])
@pytest.mark.parametrize("code", [K.BF16, K.F32])
def test_wgrad_ws_to_matches_packed_then_unpack(kind, n, h, w, cp, cq, code):
    """selunet_gemm_wgrad_ws_to (split reduction writing the reference weight layout) equals
    selunet_gemm_wgrad_ws + the unpack entry point bit for bit, for Conv2d 3x3 (halo and generic
    wgrad paths) and ConvTranspose2d operands."""
    M = n * h * w
    dt = torch.bfloat16 if code == K.BF16 else torch.float32
    p = gen(M, cp, seed=60).to(DEV).to(dt)
    if kind == "c":
        q = gen(M, cq, seed=61).to(DEV).to(dt)
        gp, gq = K.gather(n, h, w, 1, K.source(p, cp)), K.gather(n, h, w, 9, K.source(q, cq))
        kq, ni, layout = 9 * cq, cp, K.WG_CONV3X3
        out_ref = torch.empty(cp, cq, 3, 3, device=DEV)
    else:
        q = gen(4 * M, cq, seed=61).to(DEV).to(dt)  # the 2x-upsampled output gradient
        gp, gq = K.gather(n, h, w, 1, K.source(p, cp)), K.gather(n, h, w, 4, K.source(q, cq))
        kq, ni, layout = 4 * cq, cp, K.WG_CONVT
        out_ref = torch.empty(cp, cq, 2, 2, device=DEV)
    ld = K.query("selunet_wgrad_ld", kq)
    wsb = K.query("selunet_gemm_wgrad_ws_bytes", gp, gq, code)
    assert wsb > 0
    ws = torch.empty(wsb // 4, device=DEV)
    packed = torch.empty(ni, ld, device=DEV)
    K.call("selunet_gemm_wgrad_ws", gp, gq, K.ptr(packed), K.ptr(ws), wsb, code, K.stream_ptr())
    if kind == "c":
        K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), cp, cq, ld, K.ptr(out_ref), K.stream_ptr())
    else:
        K.call("selunet_unpack_convT_grad", K.ptr(packed), cp, cq, K.ptr(out_ref), K.stream_ptr())
    out = torch.full_like(out_ref, float("nan"))
    K.call("selunet_gemm_wgrad_ws_to", gp, gq, None, K.ptr(ws), wsb, layout, K.ptr(out), code, K.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)


def _bf(t):
    return t.to(torch.bfloat16).float()


def wgrad_ws(gp, gq, packed_atomic, dtype=K.BF16):
    """The deterministic split-reduced weight gradient (selunet_gemm_wgrad_ws) into a poisoned
    buffer: equal to the atomic result up to fp32 summation order, and bit-identical on a rerun."""
    outs = []
    for _ in range(2):
        wsb = K.query("selunet_gemm_wgrad_ws_bytes", gp, gq, dtype)
        assert wsb >= 0
        ws = torch.empty(max(wsb // 4, 1), device=DEV)
        out = torch.full_like(packed_atomic, float("nan"))
        K.call("selunet_gemm_wgrad_ws", gp, gq, K.ptr(out), K.ptr(ws), wsb, dtype, K.stream_ptr())
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert rel(outs[0].cpu(), packed_atomic.cpu()) < 1e-5
    return outs[0]


@pytest.mark.parametrize("cin0,cin1,cout,small,h,w", [(64, 0, 64, False, 16, 16), (64, 64, 128, False, 16, 16),
                                                      (256, 0, 512, False, 16, 16), (3, 0, 64, True, 16, 16),
                                                      (128, 0, 64, False, 20, 40), (64, 128, 64, False, 24, 17)])
@pytest.mark.parametrize("wgs", [0, 3])
def test_conv3x3_bf16_fwd_wgrad(cin0, cin1, cout, small, h, w, wgs, halo_wgs):
    """bf16 operands, fp32 accumulation: compared with fp32 torch on the same bf16-rounded data
    (sizes >= 16 take the halo-tiled kernels, incl. partial edge tiles)."""
    halo_wgs(wgs)
    n = 2
    x0 = _bf(gen(n, cin0, h, w, seed=40))
    x1 = _bf(gen(n, cin1, h, w, seed=41)) if cin1 else None
    s0, t0 = bn_fold(cin0, 42)
    cin = cin0 + cin1
    wt = _bf(gen(cout, cin, 3, 3, seed=43, scale=0.05))
    dy = _bf(gen(n, cout, h, w, seed=44))
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    if small:
        a = x0
        keep = [d(x0)]
        srcs = [K.source(keep[0], cin0, layout=1)]
    else:
        a = _bf(torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)))
        keep = [d(nhwc(x0)).bfloat16(), d(s0), d(t0)]
        srcs = [K.source(keep[0], cin0, keep[1], keep[2])]
        if cin1:
            a = torch.cat((a, x1), 1)
            keep.append(d(nhwc(x1)).bfloat16())
            srcs.append(K.source(keep[3], cin1))
    wr = wt.clone().requires_grad_()
    y = F.conv2d(a, wr, padding=1)
    (gw,) = torch.autograd.grad(y, wr, dy)
    fwd, _, kpad = pack(wt, torch.bfloat16)
    M = n * h * w
    out = torch.empty(M, cout, dtype=torch.bfloat16, device=DEV)
    ep = K.Epilogue(K.ptr(out), None, None, None, K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", K.gather(n, h, w, 9, *srcs), K.ptr(fwd), cout, kpad, ep, K.BF16, K.stream_ptr())
    assert rel(nchw(out.float().cpu(), n, h, w), y) < 1e-2
    dyd = d(nhwc(dy)).bfloat16()
    ld = K.query("selunet_wgrad_ld", 9 * cin)
    packed = torch.zeros(cout, ld, device=DEV)
    gp, gq = K.gather(n, h, w, 1, K.source(dyd, cout)), K.gather(n, h, w, 9, *srcs)
    K.call("selunet_gemm_wgrad", gp, gq, K.ptr(packed), K.BF16, K.stream_ptr())
    wgrad_ws(gp, gq, packed)
    gwd = torch.empty(cout, cin, 3, 3, device=DEV)
    K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), cout, cin, ld, K.ptr(gwd), K.stream_ptr())
    assert rel(gwd.cpu(), gw) < 1e-3  # inputs exactly bf16, fp32 accumulation


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 4, 6, 256, 128), (4, 16, 24, 128, 64), (3, 10, 14, 512, 256),
                                             (2, 6, 10, 64, 64), (2, 5, 64, 256, 128), (1, 3, 128, 128, 64)])
def test_convT_bf16_wgrad(n, h, w, cin, cout):
    """The 256-column tiles (512 threads; 256 x 256 and 128 x 256) with several pixel splits and a ragged
    last one, and the 128-column kernel (64 x 64); w % 64 == 0: one dU pixel decode per 64-pixel stage."""
    x = _bf(gen(n, cin, h, w, seed=45))
    wt = gen(cin, cout, 2, 2, seed=46, scale=0.05).requires_grad_()
    y = F.conv_transpose2d(x, wt, stride=2)
    dy = _bf(gen(*y.shape, seed=47))
    (gw,) = torch.autograd.grad(y, wt, dy)
    xd = nhwc(x).to(DEV).bfloat16()
    dud = nhwc(dy).to(DEV).bfloat16()
    ld = K.query("selunet_wgrad_ld", 4 * cout)
    packed = torch.zeros(cin, ld, device=DEV)
    gp, gq = K.gather(n, h, w, 1, K.source(xd, cin)), K.gather(n, h, w, 4, K.source(dud, cout))
    K.call("selunet_gemm_wgrad", gp, gq, K.ptr(packed), K.BF16, K.stream_ptr())
    wgrad_ws(gp, gq, packed)
    gwd = torch.empty(cin, cout, 2, 2, device=DEV)
    K.call("selunet_unpack_convT_grad", K.ptr(packed), cin, cout, K.ptr(gwd), K.stream_ptr())
    assert rel(gwd.cpu(), gw) < 1e-3


@pytest.mark.parametrize("dt,cin,n,h,w", [(torch.float32, 3, 2, 32, 32), (torch.float32, 2, 1, 20, 40),
                                          (torch.bfloat16, 3, 2, 32, 48), (torch.bfloat16, 3, 3, 64, 64)])
def test_first_conv_fwd_and_wgrad(dt, cin, n, h, w):
    """encoder_layer_1_1 (model.py:29) straight from the NCHW fp32 input: forward with BN column
    statistics, and the weight gradient through the row slab."""
    x = gen(n, cin, h, w, seed=50)
    wt = gen(64, cin, 3, 3, seed=51, scale=0.2)
    ref = F.conv2d(x, wt, padding=1)
    tol = TOL if dt == torch.float32 else 1e-2
    xd, wd = x.to(DEV).contiguous(), wt.to(DEV).contiguous()
    fwd = torch.empty(64, 32, dtype=dt, device=DEV)
    K.call("selunet_pack_conv3x3", K.ptr(wd), 64, cin, 32, K.ptr(fwd), None, K.dtype_code(dt), K.stream_ptr())
    M = n * h * w
    y = torch.empty(M, 64, dtype=dt, device=DEV)
    rows = K.query("selunet_first_conv_rows", n, h, w)
    stats = torch.empty(rows, 2, 64, device=DEV)
    K.call("selunet_first_conv_fwd", K.ptr(xd), n, cin, h, w, K.ptr(fwd), K.ptr(y), K.ptr(stats), K.dtype_code(dt),
           K.stream_ptr())
    assert rel(nchw(y.float().cpu(), n, h, w), ref) < tol
    r64 = ref.double().permute(1, 0, 2, 3).reshape(64, -1)
    st = stats.double().sum(0).cpu()
    assert rel(st[0], r64.sum(1)) < tol and rel(st[1], (r64 * r64).sum(1)) < tol
    # weight gradient
    dy = gen(n, 64, h, w, seed=52)
    dyq = dy.to(dt).float()  # what the kernel sees
    ref_w = torch.nn.grad.conv2d_weight(x, wt.shape, dyq, padding=1)
    dyd = nhwc(dy).to(dt).to(DEV)
    wrows = K.query("selunet_first_conv_wgrad_rows", n, h, w)
    slab = torch.empty(wrows, 64, 32, device=DEV)
    K.call("selunet_first_conv_wgrad", K.ptr(xd), n, cin, h, w, K.ptr(dyd), K.ptr(slab), K.dtype_code(dt),
           K.stream_ptr())
    packed = slab.double().sum(0).float().contiguous()
    gw = torch.empty(64, cin, 3, 3, device=DEV)
    K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), 64, cin, 32, K.ptr(gw), K.stream_ptr())
    assert rel(gw.cpu(), ref_w) < (TOL if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt,cin,n,h,w", [(torch.float32, 3, 2, 32, 32), (torch.float32, 2, 1, 20, 40),
                                          (torch.bfloat16, 3, 2, 32, 48)])
def test_first_conv_wgrad_bn_fused(dt, cin, n, h, w):
    """selunet_first_conv_wgrad_bn (encoder_layer_1_1's BN+ReLU backward formed while staging) against
    selunet_bn_bwd_apply + selunet_first_conv_wgrad on the same dA, y and coefficients: the same dy per
    element, so the same partial sums (fp32: to rounding of the MFMA order; bf16: dy rounded alike)."""
    M, co = n * h * w, 64
    x = gen(n, cin, h, w, seed=70).to(DEV).contiguous()
    dz = gen(M, co, seed=71).to(dt).to(DEV)
    y = gen(M, co, seed=72).to(dt).to(DEV)
    sc, sh = (gen(co, seed=73).abs() + 0.5).to(DEV), (gen(co, seed=74) * 0.3).to(DEV)
    mean, invstd = (gen(co, seed=75) * 0.1).to(DEV), (gen(co, seed=76).abs() + 0.5).to(DEV)
    coef = (gen(3, co, seed=77) * 0.2).to(DEV).contiguous()
    dy = torch.empty(M, co, dtype=dt, device=DEV)
    K.call("selunet_bn_bwd_apply", K.ptr(dz), K.ptr(y), M, co, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
           K.ptr(coef), K.ptr(dy), K.dtype_code(dt), K.stream_ptr())
    rows = K.query("selunet_first_conv_wgrad_rows", n, h, w)
    ref, got = torch.empty(rows, 64, 32, device=DEV), torch.empty(rows, 64, 32, device=DEV)
    K.call("selunet_first_conv_wgrad", K.ptr(x), n, cin, h, w, K.ptr(dy), K.ptr(ref), K.dtype_code(dt), K.stream_ptr())
    K.call("selunet_first_conv_wgrad_bn", K.ptr(x), n, cin, h, w, K.ptr(dz), K.ptr(y), K.ptr(sc), K.ptr(sh),
           K.ptr(mean), K.ptr(invstd), K.ptr(coef), K.ptr(got), K.dtype_code(dt), K.stream_ptr())
    torch.cuda.synchronize()
    r, g = ref.double().sum(0).cpu(), got.double().sum(0).cpu()
    assert rel(g, r) < (1e-6 if dt == torch.float32 else 1e-5)


@pytest.mark.parametrize("cin0,cin1,cout,n,h,w", [
    (128, 0, 128, 2, 20, 72),    # partial tiles in both directions
    (64, 0, 64, 2, 40, 36),      # one channel chunk: weights-resident persistent kernel
    (64, 0, 128, 3, 24, 24),     # one chunk, two 64-column tiles
    (128, 128, 256, 1, 33, 40),  # two sources (torch.cat), two column tiles
    (256, 0, 512, 2, 32, 32),    # four chunks, four column tiles
])
@pytest.mark.parametrize("wgs", [0, 3])
@pytest.mark.parametrize("variant", BF16_VARIANTS)
def test_conv3x3_bf16_persist_fwd_stats(cin0, cin1, cout, n, h, w, wgs, variant, halo_wgs, kernel_option):
    """bf16 multi-chunk 3x3 forward on the persistent halo kernel with the BN statistics epilogue;
    wgs = 3 makes every workgroup walk several tiles; variant: a kernel-selection option set for the test."""
    halo_wgs(wgs)
    kernel_option(variant)
    x0 = _bf(gen(n, cin0, h, w, seed=60))
    x1 = _bf(gen(n, cin1, h, w, seed=61)) if cin1 else None
    s0, t0 = bn_fold(cin0, 62)
    wt = _bf(gen(cout, cin0 + cin1, 3, 3, seed=63, scale=0.05))
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    a = _bf(torch.relu(x0 * s0.view(1, -1, 1, 1) + t0.view(1, -1, 1, 1)))
    keep = [d(nhwc(x0)).bfloat16(), d(s0), d(t0)]
    srcs = [K.source(keep[0], cin0, keep[1], keep[2])]
    if cin1:
        a = torch.cat((a, x1), 1)
        keep.append(d(nhwc(x1)).bfloat16())
        srcs.append(K.source(keep[3], cin1))
    ref = F.conv2d(a, wt, padding=1)
    fwd, _, kpad = pack(wt, torch.bfloat16)
    g = K.gather(n, h, w, 9, *srcs)
    M = n * h * w
    out = torch.empty(M, cout, dtype=torch.bfloat16, device=DEV)
    rows = K.query("selunet_gemm_stats_rows", g, cout, K.BF16)
    stats = torch.empty(rows, 2, cout, device=DEV)
    ep = K.Epilogue(K.ptr(out), None, None, K.ptr(stats), K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", g, K.ptr(fwd), cout, kpad, ep, K.BF16, K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(nchw(out.float().cpu(), n, h, w), ref) < 1e-2
    st = stats.cpu().double().sum(0)
    r = ref.double().permute(1, 0, 2, 3).reshape(cout, -1)
    assert rel(st[0], r.sum(1)) < 1e-3 and rel(st[1], (r * r).sum(1)) < 1e-3


@pytest.mark.parametrize("cin,cout,split,h,w", [(256, 128, 0, 20, 40), (256, 128, 128, 16, 64),
                                                (512, 256, 256, 32, 32), (64, 64, 0, 20, 40),
                                                (128, 64, 64, 24, 40)])
@pytest.mark.parametrize("wgs", [0, 3])
@pytest.mark.parametrize("variant", BF16_VARIANTS)
def test_conv3x3_bf16_persist_dgrad(cin, cout, split, h, w, wgs, variant, halo_wgs, kernel_option):
    """bf16 data gradient on the persistent halo kernel: plain with the producer's BN-backward sums,
    and the torch.cat split with the ConvTranspose2d bias column sums."""
    halo_wgs(wgs)
    kernel_option(variant)
    n = 2
    wt = _bf(gen(cout, cin, 3, 3, seed=64, scale=0.05))
    dy = _bf(gen(n, cout, h, w, seed=65))
    x = gen(n, cin, h, w, seed=66).requires_grad_()
    (ref,) = torch.autograd.grad(F.conv2d(x, wt, padding=1), x, dy)
    _, dg, _ = pack(wt, torch.bfloat16)
    dyd = nhwc(dy).to(DEV).bfloat16()
    M = n * h * w
    g = K.gather(n, h, w, 9, K.source(dyd, cout))
    rows = K.query("selunet_gemm_stats_rows", g, cin, K.BF16)
    if split:
        d0 = torch.empty(M, split, dtype=torch.bfloat16, device=DEV)
        d1 = torch.empty(M, cin - split, dtype=torch.bfloat16, device=DEV)
        colsum = torch.empty(rows, split, device=DEV)
        ep = K.Epilogue(K.ptr(d0), K.ptr(d1), None, None, K.EP_SPLIT, split, K.ptr(colsum))
        K.call("selunet_gemm_gather", g, K.ptr(dg), cin, 9 * cout, ep, K.BF16, K.stream_ptr())
        torch.cuda.synchronize()
        got = torch.cat((nchw(d0.float().cpu(), n, h, w), nchw(d1.float().cpu(), n, h, w)), 1)
        assert rel(colsum.double().sum(0).cpu(), d0.double().sum(0).cpu()) < 1e-5
    else:
        dx = torch.empty(M, cin, dtype=torch.bfloat16, device=DEV)
        yprev = gen(M, cin, seed=67).to(DEV).bfloat16()
        sc, sh = (gen(cin, seed=68).abs() + 0.5).to(DEV), (gen(cin, seed=69) * 0.3).to(DEV)
        mean, invstd = (gen(cin, seed=70) * 0.1).to(DEV), (gen(cin, seed=71).abs() + 0.5).to(DEV)
        slab = torch.empty(rows, 3, cin, device=DEV)
        ep = K.Epilogue(K.ptr(dx), None, None, None, K.EP_PLAIN, 0)
        ep.bnb = K.BnBwdStats(K.ptr(yprev), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
        K.call("selunet_gemm_gather", g, K.ptr(dg), cin, 9 * cout, ep, K.BF16, K.stream_ptr())
        torch.cuda.synchronize()
        got = nchw(dx.float().cpu(), n, h, w)
        check_bnb_sums(slab.cpu(), dx.float().cpu(), yprev.float().cpu(), sc.cpu(), sh.cpu(), mean.cpu(),
                       invstd.cpu(), tol=1e-4)
    assert rel(got, ref) < 1e-2


@pytest.mark.parametrize("c", [64, 256])
def test_bn_adaptive_centered_variance(c):
    """selunet_bn_centered_partials_adaptive (fp32 BatchNorm variance, engine default): channels
    whose mean^2 exceeds ratio x the one-pass variance are re-read (centered sums), the others reuse
    the one-pass variance exactly. Against the fp64 batch statistics of y: mean within 1e-6 of the
    scale, variance within 1e-5 relative on the re-read groups (where the one-pass E[y^2] - mean^2
    is off by ~eps * mean^2 / var) and within 1e-5 on the others; running statistics updated once."""
    M = 50000
    g = torch.Generator().manual_seed(11)
    means = torch.where(torch.arange(c) % 8 < 4, 300.0, 0.3)  # groups of 4: large / small mean^2 / var
    # near-constant channels (var 1e-9, far below eps_bn) with a mean shift whose square is
    # below eps_bn but far above var: the one-pass variance is ~5e-4 off, so they must be re-read too
    tiny = torch.arange(c) % 16 >= 12
    means = torch.where(tiny, 3e-3, means)
    stds = torch.where(tiny, 3.16e-5, 1.0)
    y = (torch.randn(M, c, generator=g, dtype=torch.float64) * stds + means).float().to(DEV)
    rows = K.query("selunet_bn_centered_rows", M)
    slab1 = torch.zeros(1, 2, c, device=DEV)
    slab1[0, 0] = y.double().sum(0).float()          # the conv epilogue's one-pass sums (fp32 slab)
    slab1[0, 1] = (y.double() ** 2).sum(0).float()
    ws = torch.empty(K.query("selunet_reduce_ws_bytes", 2 * c) // 8, dtype=torch.float64, device=DEV)
    gamma, beta = torch.ones(c, device=DEV), torch.zeros(c, device=DEV)
    outs = []
    for adaptive in (True, False):
        mean, invstd, scale, shift = (torch.empty(c, device=DEV) for _ in range(4))
        uvar = torch.zeros(c, device=DEV)
        K.call("selunet_bn_stats_finalize", K.ptr(slab1), 1, K.ptr(ws), None, M, c, None, K.ptr(gamma),
               K.ptr(beta), None, K.ptr(uvar), None, 1.0, 1e-5, K.ptr(mean), K.ptr(invstd), K.ptr(scale),
               K.ptr(shift), K.stream_ptr())
        slab2 = torch.empty(rows, 2, c, device=DEV)
        if adaptive:
            K.call("selunet_bn_centered_partials_adaptive", K.ptr(y), M, c, K.ptr(mean), K.ptr(uvar), 1.0,
                   K.ptr(slab2), K.F32, K.stream_ptr())
        else:
            K.call("selunet_bn_centered_partials", K.ptr(y), M, c, K.ptr(mean), K.ptr(slab2), K.F32,
                   K.stream_ptr())
        rm, rv = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)  # zero: rv is 0.1 x the unbiased var
        nbt = torch.zeros((), dtype=torch.int64, device=DEV)
        K.call("selunet_bn_stats_finalize_centered", K.ptr(slab2), rows, K.ptr(ws), None, M, c, K.ptr(mean), None,
               K.ptr(gamma), K.ptr(beta), K.ptr(rm), K.ptr(rv), K.ptr(nbt), 0.1, 1e-5, K.ptr(mean), K.ptr(invstd),
               K.ptr(scale), K.ptr(shift), K.stream_ptr())
        torch.cuda.synchronize()
        outs.append((mean.cpu().double(), invstd.cpu().double(), rv.cpu().double(), int(nbt)))
    yd = y.cpu().double()
    m64, v64 = yd.mean(0), yd.var(0, unbiased=False)
    for mean, invstd, rv, nbt in outs:
        assert nbt == 1
        assert ((mean - m64).abs() / (m64.abs() + 1)).max() < 1e-6
        var = 1.0 / invstd ** 2 - 1e-5  # (fp32 invstd: var is resolved to ~1e-7 of var + eps_bn)
        assert ((var - v64).abs() / v64.clamp(min=1e-5)).max() < 1e-5
        want = 0.1 * v64 * M / (M - 1)
        assert ((rv - want).abs() / want).max() < 2e-5  # running variance, relative (incl. the tiny channels)
