"""bf16 ConvTranspose2d forward / data gradient on the resident-weight kernels (convt_bf16.hip, behind
selunet_gemm_gather with SELUNET_BF16; model.py:44-45, 51-52, 57-58) against torch in fp32 on the same
bf16 operands.

Tolerance: the reference is computed from the identical bf16-rounded operands (the producer's BN+ReLU
applied and rounded to bf16 as the kernel's stager does), accumulated in fp32 / fp64, so the kernel
differs only by its fp32 accumulation order and the final bf16 rounding of the output: 8e-3 of the
tensor's max magnitude (two bf16 half-ulps at the top of the range). The BN-backward sums are checked
against the sums of the kernel's own bf16 output (tests/test_gpu_kernels.check_bnb_sums)."""
import pytest
import torch
import torch.nn.functional as F

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from tests.test_gpu_kernels import bn_fold, check_bnb_sums, gen, nchw, nhwc, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 8e-3
BF = torch.bfloat16


@pytest.fixture
def convt_ring():
    """Set SELUNET_OPT_CONVT_RING for one test (0: the resident-weight kernels for unpool3 / unpool2 too)."""
    prev = []

    def setter(mode):
        prev.append(K.set_option("CONVT_RING", mode))
    yield setter
    for v in prev[:1]:
        K.set_option("CONVT_RING", v)


def pack_convT_bf16(wt):
    """selunet_pack_convT in bf16: fwd [4*co][ci], dgrad [ci][4*co]."""
    ci, co = wt.shape[:2]
    wd = wt.to(DEV).float().contiguous()
    fwd = torch.empty(4 * co, ci, dtype=BF, device=DEV)
    dg = torch.empty(ci, 4 * co, dtype=BF, device=DEV)
    K.call("selunet_pack_convT", K.ptr(wd), ci, co, K.ptr(fwd), K.ptr(dg), K.BF16, K.stream_ptr())
    return fwd, dg


@pytest.mark.parametrize("cin,cout,n,h,w", [
    (128, 64, 2, 9, 64),     # unpool1 (K = 128: all 256 columns resident), partial last tile
    (256, 128, 2, 5, 64),    # unpool2 (K = 256, two column blocks)
    (512, 256, 2, 4, 32),    # unpool3 (K = 512, eight column blocks)
    (128, 64, 4, 40, 256),   # several tiles per workgroup
])
def test_convT_bf16_fwd(cin, cout, n, h, w, convt_ring):
    convt_ring(0)  # (the resident-weight kernel; the ring kernel: test_convT_bf16_ring_matches_resident)
    x = gen(n, cin, h, w, seed=61).to(BF)
    s, t = bn_fold(cin, 62)
    a = torch.relu(x.float() * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1)).to(BF)  # the stager's bf16 operand
    wt = gen(cin, cout, 2, 2, seed=63, scale=0.05).to(BF)
    b = gen(cout, seed=64)
    ref = F.conv_transpose2d(a.double(), wt.double(), b.double(), stride=2)
    fwd, _ = pack_convT_bf16(wt.float())
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    xd, sd, td, bd = d(nhwc(x)), d(s), d(t), d(b)
    g = K.gather(n, h, w, 1, K.source(xd, cin, sd, td))
    assert K.query("selunet_gemm_kernel_name", g, None, 4 * cout, K.EP_SCATTER2X, K.BF16) == b"convt<bf16>"
    up = torch.full((n * 2 * h * 2 * w, cout), float("nan"), dtype=BF, device=DEV)
    ep = K.Epilogue(K.ptr(up), None, K.ptr(bd), None, K.EP_SCATTER2X, 0)
    K.call("selunet_gemm_gather", g, K.ptr(fwd), 4 * cout, cin, ep, K.BF16, K.stream_ptr())
    torch.cuda.synchronize()
    got = nchw(up.float().cpu(), n, 2 * h, 2 * w)
    assert not torch.isnan(got).any()
    assert rel(got, ref) < TOL


@pytest.mark.parametrize("cin,cout,n,h,w", [
    (128, 64, 2, 9, 64),     # unpool1 (K = 256, 128 columns)
    (256, 128, 2, 5, 64),    # unpool2 (K = 512, two column blocks)
    (512, 256, 2, 4, 32),    # unpool3 (K = 1024, eight column blocks of 64)
    (128, 64, 4, 72, 256),   # several tiles per workgroup
])
def test_convT_bf16_dgrad(cin, cout, n, h, w, convt_ring):
    convt_ring(0)
    x = gen(n, cin, h, w, seed=65).double().requires_grad_()
    wt = gen(cin, cout, 2, 2, seed=66, scale=0.05).to(BF)
    y = F.conv_transpose2d(x, wt.double(), None, stride=2)
    dy = (gen(*y.shape, seed=67) * 1e-3).to(BF)
    (ref,) = torch.autograd.grad(y, (x,), dy.double())
    _, dg = pack_convT_bf16(wt.float())
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    dud = d(nhwc(dy))
    M = n * h * w
    yprev = gen(M, cin, seed=68).to(BF).to(DEV)
    sc, sh = (gen(cin, seed=69).abs() + 0.5).to(DEV), (gen(cin, seed=70) * 0.3).to(DEV)
    mean, invstd = (gen(cin, seed=71) * 0.1).to(DEV), (gen(cin, seed=72).abs() + 0.5).to(DEV)
    g4 = K.gather(n, h, w, 4, K.source(dud, cout))
    assert K.query("selunet_gemm_kernel_name", g4, None, cin, K.EP_PLAIN, K.BF16) == b"convt_dgrad<bf16>"
    rows = K.query("selunet_gemm_stats_rows", g4, cin, K.BF16)
    ntb = 64 if cout == 256 else 128
    tile = 8 * (8 // (ntb // 32)) * 32
    assert rows == min(-(-M // tile), 256 // (cin // ntb))  # the resident-weight kernel's workgroup rows
    slab = torch.full((rows, 3, cin), float("nan"), device=DEV)
    da = torch.full((M, cin), float("nan"), dtype=BF, device=DEV)
    ep = K.Epilogue(K.ptr(da), None, None, None, K.EP_PLAIN, 0)
    ep.bnb = K.BnBwdStats(K.ptr(yprev), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
    K.call("selunet_gemm_gather", g4, K.ptr(dg), cin, 4 * cout, ep, K.BF16, K.stream_ptr())
    torch.cuda.synchronize()
    assert rel(nchw(da.float().cpu(), n, h, w), ref) < TOL
    check_bnb_sums(slab, da.float(), yprev.float(), sc, sh, mean, invstd, tol=1e-4)
    # without the statistics: same values
    da2 = torch.empty_like(da)
    ep = K.Epilogue(K.ptr(da2), None, None, None, K.EP_PLAIN, 0)
    K.call("selunet_gemm_gather", g4, K.ptr(dg), cin, 4 * cout, ep, K.BF16, K.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(da2, da)


def test_convT_bf16_rejects_sums_on_other_epilogues():
    """A data-gradient operand the statistics query sizes for the resident-weight kernel cannot take a
    statistics epilogue the kernel does not run (SPLIT / bias): refused on the host."""
    n, h, w, cin, cout = 1, 2, 32, 128, 64
    dud = torch.zeros(n * 4 * h * w, cout, dtype=BF, device=DEV)
    _, dg = pack_convT_bf16(torch.zeros(cin, cout, 2, 2))
    g4 = K.gather(n, h, w, 4, K.source(dud, cout))
    out = torch.empty(n * h * w, cin, dtype=BF, device=DEV)
    slab = torch.empty(64, 3, cin, device=DEV)
    ep = K.Epilogue(K.ptr(out), None, K.ptr(torch.zeros(cin, device=DEV)), None, K.EP_PLAIN, 0)
    ep.bnb = K.BnBwdStats(K.ptr(out), K.ptr(slab), K.ptr(slab), K.ptr(slab), K.ptr(slab), K.ptr(slab))
    with pytest.raises(RuntimeError):
        K.call("selunet_gemm_gather", g4, K.ptr(dg), cin, 4 * cout, ep, K.BF16, K.stream_ptr())


def _bf16_pair(cin, cout, n, h, w, seed):
    x = gen(n, cin, h, w, seed=seed).to(BF)
    s, t = bn_fold(cin, seed + 1)
    wt = gen(cin, cout, 2, 2, seed=seed + 2, scale=0.05).to(BF)
    b = gen(cout, seed=seed + 3)
    dy = (gen(n, cout, 2 * h, 2 * w, seed=seed + 4) * 1e-3).to(BF)
    fwd, dg = pack_convT_bf16(wt.float())
    d = lambda t_: t_.to(DEV).contiguous()  # noqa: E731
    xd, sd, td, bd, dud = d(nhwc(x)), d(s), d(t), d(b), d(nhwc(dy))
    M = n * h * w
    up = torch.full((4 * M, cout), float("nan"), dtype=BF, device=DEV)
    ep = K.Epilogue(K.ptr(up), None, K.ptr(bd), None, K.EP_SCATTER2X, 0)
    K.call("selunet_gemm_gather", K.gather(n, h, w, 1, K.source(xd, cin, sd, td)), K.ptr(fwd), 4 * cout, cin, ep,
           K.BF16, K.stream_ptr())
    yprev = gen(M, cin, seed=seed + 5).to(BF).to(DEV)
    sc, sh = (gen(cin, seed=seed + 6).abs() + 0.5).to(DEV), (gen(cin, seed=seed + 7) * 0.3).to(DEV)
    mean, invstd = (gen(cin, seed=seed + 8) * 0.1).to(DEV), (gen(cin, seed=seed + 9).abs() + 0.5).to(DEV)
    g4 = K.gather(n, h, w, 4, K.source(dud, cout))
    rows = K.query("selunet_gemm_stats_rows", g4, cin, K.BF16)
    slab = torch.full((rows, 3, cin), float("nan"), device=DEV)
    da = torch.full((M, cin), float("nan"), dtype=BF, device=DEV)
    ep = K.Epilogue(K.ptr(da), None, None, None, K.EP_PLAIN, 0)
    ep.bnb = K.BnBwdStats(K.ptr(yprev), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(slab))
    K.call("selunet_gemm_gather", g4, K.ptr(dg), cin, 4 * cout, ep, K.BF16, K.stream_ptr())
    torch.cuda.synchronize()
    return dict(x=x, s=s, t=t, wt=wt, b=b, dy=dy, up=up, da=da, slab=slab, rows=rows, yprev=yprev, sc=sc, sh=sh,
                mean=mean, invstd=invstd)


@pytest.mark.parametrize("cin,cout,n,h,w", [
    (512, 256, 2, 32, 32),    # unpool3 (forward K 512 / N 1024, data gradient K 1024 / N 512)
    (256, 128, 1, 64, 64),    # unpool2 (K 256 / N 512, K 512 / N 256)
    (256, 128, 4, 128, 160),  # data gradient: 320 row tiles on 256 workgroups
])
def test_convT_bf16_ring_matches_resident(cin, cout, n, h, w, convt_ring):
    """The bf16 LDS-DMA ring kernel (convt_ring_bf16_kernel) computes convt_bf16_kernel's products in the same
    order with the same rounding: outputs bit-identical with SELUNET_OPT_CONVT_RING on and off; against torch
    on the same bf16 operands; BN-backward sums against the sums of its own output (one slab row per ring
    workgroup)."""
    convt_ring(0)
    off = _bf16_pair(cin, cout, n, h, w, seed=90)
    convt_ring(2)
    on = _bf16_pair(cin, cout, n, h, w, seed=90)
    assert torch.equal(on["up"], off["up"])
    assert torch.equal(on["da"], off["da"])
    M = n * h * w
    assert on["rows"] == min(M // 256, max(1, 256 // (cin // 256)))  # the ring kernel's workgroup rows
    a = torch.relu(on["x"].float() * on["s"].view(1, -1, 1, 1) + on["t"].view(1, -1, 1, 1)).to(BF)
    ref = F.conv_transpose2d(a.double(), on["wt"].double(), on["b"].double(), stride=2)
    assert rel(nchw(on["up"].float().cpu(), n, 2 * h, 2 * w), ref) < TOL
    check_bnb_sums(on["slab"], on["da"].float(), on["yprev"].float(), on["sc"], on["sh"], on["mean"], on["invstd"],
                   tol=1e-4)
