"""BatchNorm-backward apply with dA formed on the fly (selunet_bn_bwd_apply_heads / _pool) against the
unfused pair it replaces: the producer writing dA (selunet_heads_bwd / selunet_maxpool2_bwd) and
selunet_bn_bwd_apply_amax reading it. The producers' sums-only mode (dz = NULL) must write the same
BN-backward and head-weight sums, and the fused apply the same dy and range word, bit for bit (same
arithmetic, dA rounded to the tensor dtype as stored) — in fp32 and bf16."""
import ctypes

import pytest
import torch

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from tests.test_gpu_kernels import gen

pytestmark = pytest.mark.gpu
DEV = "cuda"


def coefs(c, seed):
    sc, sh = (gen(c, seed=seed).abs() + 0.5).to(DEV), (gen(c, seed=seed + 1) * 0.3).to(DEV)
    mean, invstd = (gen(c, seed=seed + 2) * 0.1).to(DEV), (gen(c, seed=seed + 3).abs() + 0.5).to(DEV)
    coef = (gen(3, c, seed=seed + 4) * 0.5).to(DEV).contiguous()
    return sc, sh, mean, invstd, coef


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nh", [1, 3])
def test_apply_heads_equals_unfused(dt, nh):
    m = 3 * 4096 + 77  # ragged tail
    code = K.dtype_code(dt)
    y = gen(m, 64, seed=1).to(dt).to(DEV)
    sc, sh, mean, invstd, coef = coefs(64, 10)
    w = (gen(3, 64, seed=2) * 0.2).to(DEV).contiguous()
    g = [(gen(m, seed=3 + i) * 1e-3).to(DEV) for i in range(3)]
    gp = [K.ptr(g[i]) if i < nh else None for i in range(3)]
    rows = K.query("selunet_channel_slab_rows", m)
    res = []
    for fused in (False, True):
        slab = torch.full((rows, nh * 65), float("nan"), device=DEV)
        bslab = torch.full((rows, 3, 64), float("nan"), device=DEV)
        bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(bslab))
        dz = None if fused else torch.empty(m, 64, dtype=dt, device=DEV)
        K.call("selunet_heads_bwd", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(w), nh, *gp, K.ptr(dz), K.ptr(slab), bnb,
               code, K.stream_ptr())
        dy = torch.empty(m, 64, dtype=dt, device=DEV)
        am = torch.zeros(1, device=DEV)
        if fused:
            K.call("selunet_bn_bwd_apply_heads", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
                   K.ptr(coef), K.ptr(w), nh, *gp, K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        else:
            K.call("selunet_bn_bwd_apply_amax", K.ptr(dz), K.ptr(y), m, 64, K.ptr(sc), K.ptr(sh), K.ptr(mean),
                   K.ptr(invstd), K.ptr(coef), K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        torch.cuda.synchronize()
        res.append((slab.cpu(), bslab.cpu(), dy.float().cpu(), am.item()))
    (s0, b0, d0, a0), (s1, b1, d1, a1) = res
    assert torch.equal(s0, s1) and torch.equal(b0, b1)
    assert torch.equal(d0, d1)
    assert a0 == a1 and (dt != torch.float32 or a0 == d0.abs().max().item())  # (the word is max|dy| before rounding)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c,skip", [(64, True), (128, True), (256, False)])
def test_apply_pool_equals_unfused(dt, c, skip):
    n, h, w = 2, 18, 36
    code = K.dtype_code(dt)
    m = n * h * w
    y = ((gen(m, c, seed=21) * 2).round() / 2).to(dt).to(DEV)  # coarse values: ties inside the windows
    sc, sh, mean, invstd, coef = coefs(c, 30)
    dp = (gen(m // 4, c, seed=22) * 1e-2).to(dt).to(DEV)
    ds = (gen(m, c, seed=23) * 1e-2).to(dt).to(DEV) if skip else None
    rows = K.query("selunet_maxpool2_bwd_slab_rows", n, h, w, c)
    res = []
    for fused in (False, True):
        bslab = torch.full((rows, 3, c), float("nan"), device=DEV)
        bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(bslab))
        dz = None if fused else torch.empty(m, c, dtype=dt, device=DEV)
        K.call("selunet_maxpool2_bwd", K.ptr(y), n, h, w, c, K.ptr(sc), K.ptr(sh), K.ptr(dp), K.ptr(ds), K.ptr(dz),
               bnb, code, K.stream_ptr())
        dy = torch.empty(m, c, dtype=dt, device=DEV)
        am = torch.zeros(1, device=DEV)
        if fused:
            K.call("selunet_bn_bwd_apply_pool", K.ptr(y), n, h, w, c, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
                   K.ptr(coef), K.ptr(dp), K.ptr(ds), K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        else:
            K.call("selunet_bn_bwd_apply_amax", K.ptr(dz), K.ptr(y), m, c, K.ptr(sc), K.ptr(sh), K.ptr(mean),
                   K.ptr(invstd), K.ptr(coef), K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        torch.cuda.synchronize()
        res.append((bslab.cpu(), dy.float().cpu(), am.item()))
    (b0, d0, a0), (b1, d1, a1) = res
    assert torch.equal(b0, b1)
    assert torch.equal(d0, d1)
    assert a0 == a1 and (dt != torch.float32 or a0 == d0.abs().max().item())  # (the word is max|dy| before rounding)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_apply_heads_planes_equals_unfused(dt):
    """The CE UNet's N-output heads (selunet_heads_bwd_planes / selunet_bn_bwd_apply_heads_planes): 2 images,
    outputs of 2 + 2 + 2 channels as NCHW planes."""
    n, hw, nk = 2, 48 * 40, 6
    m = n * hw
    code = K.dtype_code(dt)
    y = gen(m, 64, seed=81).to(dt).to(DEV)
    sc, sh, mean, invstd, coef = coefs(64, 90)
    w = (gen(8, 64, seed=82) * 0.2).to(DEV).contiguous()
    g = (gen(3, n, 2, hw, seed=83) * 1e-3).to(DEV).contiguous()  # three [N, 2, H*W] gradient tensors
    hp = K.HeadPlanes()
    hp.n, hp.hw = nk, hw
    row_len = 0
    for k in range(nk):
        t, j = divmod(k, 2)
        hp.plane[k] = g[t].data_ptr() + j * hw * 4
        hp.img_stride[k] = 2 * hw
        hp.w_off[k] = k * 65
        hp.b_off[k] = k * 65 + 64
        row_len = (k + 1) * 65
    hp.row_len = row_len
    rows = K.query("selunet_channel_slab_rows", m)
    res = []
    for fused in (False, True):
        slab = torch.full((rows, row_len), float("nan"), device=DEV)
        bslab = torch.full((rows, 3, 64), float("nan"), device=DEV)
        bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(bslab))
        dz = None if fused else torch.empty(m, 64, dtype=dt, device=DEV)
        K.call("selunet_heads_bwd_planes", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(w), hp, K.ptr(dz), K.ptr(slab), bnb,
               code, K.stream_ptr())
        dy = torch.empty(m, 64, dtype=dt, device=DEV)
        am = torch.zeros(1, device=DEV)
        if fused:
            K.call("selunet_bn_bwd_apply_heads_planes", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
                   K.ptr(coef), K.ptr(w), hp, K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        else:
            K.call("selunet_bn_bwd_apply_amax", K.ptr(dz), K.ptr(y), m, 64, K.ptr(sc), K.ptr(sh), K.ptr(mean),
                   K.ptr(invstd), K.ptr(coef), K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        torch.cuda.synchronize()
        res.append((slab.cpu(), bslab.cpu(), dy.float().cpu(), am.item()))
    (s0, b0, d0, a0), (s1, b1, d1, a1) = res
    assert torch.equal(s0, s1) and torch.equal(b0, b1)
    assert torch.equal(d0, d1)
    assert a0 == a1


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [64, 128, 256, 512])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_apply_forms_equal(dt, c, form):
    """The apply kernel's alternative forms (SELUNET_OPT_APPLY_U8: 8 channels x 8 pixels, 4 contiguous
    channels x 8 / 16 pixels) against the default form, bit for bit, ragged pixel count."""
    m = 4096 * 3 + 5
    code = K.dtype_code(dt)
    y = gen(m, c, seed=41).to(dt).to(DEV)
    dz = (gen(m, c, seed=42) * 1e-2).to(dt).to(DEV)
    sc, sh, mean, invstd, coef = coefs(c, 50)
    res = []
    for f in (0, form):
        prev = K.set_option("APPLY_U8", f)
        dy = torch.full((m, c), float("nan"), dtype=dt, device=DEV)
        am = torch.zeros(1, device=DEV)
        K.call("selunet_bn_bwd_apply_amax", K.ptr(dz), K.ptr(y), m, c, K.ptr(sc), K.ptr(sh), K.ptr(mean),
               K.ptr(invstd), K.ptr(coef), K.ptr(dy), K.ptr(am), code, K.stream_ptr())
        torch.cuda.synchronize()
        K.set_option("APPLY_U8", prev)
        res.append((dy.float().cpu(), am.item()))
    assert torch.equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]


def test_sums_only_needs_the_sums():
    """dz = NULL without a BN-backward slab would compute nothing: refused on the host."""
    y = torch.zeros(64, 64, device=DEV)
    sc = torch.ones(64, device=DEV)
    with pytest.raises(RuntimeError):
        K.call("selunet_maxpool2_bwd", K.ptr(y), 1, 8, 8, 64, K.ptr(sc), K.ptr(sc), K.ptr(y), None, None, None, K.F32,
               K.stream_ptr())


def _bn_state(m, c, seed):
    """y with its real batch statistics (the Samuelson bound of selunet_bn_bwd_stats_finalize_bound holds
    for those only), the forward's folded scale / shift, and a dA."""
    g = torch.Generator().manual_seed(seed)
    y = (torch.randn(m, c, generator=g, dtype=torch.float64) * (torch.rand(c, generator=g, dtype=torch.float64) + 0.2)
         + torch.randn(c, generator=g, dtype=torch.float64))
    mean, var = y.mean(0), y.var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    gamma = torch.randn(c, generator=g, dtype=torch.float64) * 0.5 + 1.0
    beta = torch.randn(c, generator=g, dtype=torch.float64) * 0.2
    sc, sh = gamma * invstd, beta - mean * gamma * invstd
    da = torch.randn(m, c, generator=g, dtype=torch.float64) * 1e-3
    f = lambda t: t.float().to(DEV).contiguous()  # noqa: E731
    return f(y), f(mean), f(invstd), f(gamma), f(sc), f(sh), f(da)


@pytest.mark.parametrize("c", [64, 256])
def test_bn_bwd_finalize_bound_covers_dy(c):
    """selunet_bn_bwd_stats_finalize_bound: the same coefficients and parameter gradients as
    selunet_bn_bwd_stats_finalize, and a range word >= max |dy| of the apply they feed."""
    m = 20000
    y, mean, invstd, gamma, sc, sh, da = _bn_state(m, c, 5)
    mask = (y * sc + sh > 0).float()
    xh = (y - mean) * invstd
    slab = torch.stack([(da * mask).sum(0), (da * mask * xh).sum(0), xh.sum(0)]).reshape(1, 3, c).contiguous()
    ws = torch.empty(K.query("selunet_reduce_ws_bytes", 3 * c) // 8, dtype=torch.float64, device=DEV)
    amax_da = da.abs().max().reshape(1).contiguous()
    outs = []
    for bound in (False, True):
        coef, dg, db, dbias = (torch.empty(3, c, device=DEV), torch.empty(c, device=DEV), torch.empty(c, device=DEV),
                               torch.empty(c, device=DEV))
        word = torch.zeros(1, device=DEV)
        if bound:
            K.call("selunet_bn_bwd_stats_finalize_bound", K.ptr(slab), 1, K.ptr(ws), None, m, c, K.ptr(gamma),
                   K.ptr(invstd), K.ptr(dg), K.ptr(db), K.ptr(dbias), K.ptr(coef), K.ptr(amax_da), K.ptr(word),
                   K.stream_ptr())
        else:
            K.call("selunet_bn_bwd_stats_finalize", K.ptr(slab), 1, K.ptr(ws), None, m, c, K.ptr(gamma), K.ptr(invstd),
                   K.ptr(dg), K.ptr(db), K.ptr(dbias), K.ptr(coef), K.stream_ptr())
        outs.append((coef.cpu(), dg.cpu(), db.cpu(), dbias.cpu(), word.item()))
    (c0, g0, b0, d0, _), (c1, g1, b1, d1, w1) = outs
    assert torch.equal(c0, c1) and torch.equal(g0, g1) and torch.equal(b0, b1) and torch.equal(d0, d1)
    dy = torch.empty(m, c, device=DEV)
    am = torch.zeros(1, device=DEV)
    K.call("selunet_bn_bwd_apply_amax", K.ptr(da), K.ptr(y), m, c, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
           K.ptr(c1.to(DEV)), K.ptr(dy), K.ptr(am), K.F32, K.stream_ptr())
    torch.cuda.synchronize()
    assert 0.0 < am.item() <= w1
    print(f"bound / max|dy| = {w1 / am.item():.1f}")


@pytest.mark.parametrize("co,ci", [(64, 64), (64, 128), (128, 128), (256, 64)])
def test_wgrad_x2_bn_equals_apply_then_wgrad(co, ci):
    """selunet_conv3x3_wgrad_x2_bn (the BN-backward apply in the weight gradient's dY staging) against
    selunet_bn_bwd_apply_amax + selunet_conv3x3_wgrad_x2: dy and max |dy| identical (same arithmetic),
    the weight gradient within split-fp16 rounding of it and of the fp64 weight gradient, although it
    stages dy with a looser range word (a bound 37x the exact max)."""
    n, h, w = 2, 20, 36  # ragged 8x8 tiles in y
    m = n * h * w
    y, mean, invstd, _, sc, sh, da = _bn_state(m, co, 7)
    coef = (gen(3, co, seed=70) * 0.5).to(DEV).contiguous()
    coef[0] = coef[0].abs() + 0.5
    x = gen(m, ci, seed=71).to(DEV)
    xsc, xsh = (gen(ci, seed=72).abs() + 0.5).to(DEV), (gen(ci, seed=73) * 0.2).to(DEV)
    xw = (torch.relu(x * xsc + xsh)).abs().max().reshape(1).contiguous()
    gq = K.gather(n, h, w, 9, K.source(x, ci, xsc, xsh, relu=True, amax=xw))
    # unfused pair
    dy0 = torch.empty(m, co, device=DEV)
    am0 = torch.zeros(1, device=DEV)
    K.call("selunet_bn_bwd_apply_amax", K.ptr(da), K.ptr(y), m, co, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
           K.ptr(coef), K.ptr(dy0), K.ptr(am0), K.F32, K.stream_ptr())
    gp0 = K.gather(n, h, w, 1, K.source(dy0, co))
    wsb = K.query("selunet_conv3x3_wgrad_x2_ws_bytes", gp0, gq)
    assert wsb > 0
    ws = torch.empty(wsb // 4, device=DEV)
    dw0 = torch.empty(co, ci, 3, 3, device=DEV)
    K.call("selunet_conv3x3_wgrad_x2", gp0, gq, K.ptr(ws), wsb, K.ptr(dw0), K.ptr(am0), K.ptr(xw), None, K.stream_ptr())
    torch.cuda.synchronize()
    # fused (static walk, then SELUNET_OPT_TILE_QUEUE bit 1: tiles from ticket counters — dy and max |dy| are the
    # same element-wise arithmetic, the weight gradient the same sum in another order)
    bound = (am0 * 37.0).contiguous()
    gp1 = K.gather(n, h, w, 1, K.source(da, co))
    bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), None)
    fused = []
    prev = K.set_option("TILE_QUEUE", 0)
    try:
        for tq in (0, 2):
            K.set_option("TILE_QUEUE", tq)
            dy1 = torch.full((m, co), float("nan"), device=DEV)
            am1 = torch.zeros(1, device=DEV)
            dw1 = torch.empty(co, ci, 3, 3, device=DEV)
            K.call("selunet_conv3x3_wgrad_x2_bn", gp1, gq, K.ptr(ws), wsb, K.ptr(dw1), K.ptr(bound), K.ptr(xw), None,
                   bnb, K.ptr(coef), K.ptr(dy1), K.ptr(am1), K.stream_ptr())
            torch.cuda.synchronize()
            assert torch.equal(dy1.cpu(), dy0.cpu()), tq
            assert am1.item() == am0.item(), tq
            fused.append(dw1.cpu())
    finally:
        K.set_option("TILE_QUEUE", prev)
    assert float((fused[1].double() - fused[0].double()).norm() / fused[0].double().norm()) < 1e-6
    dw1 = fused[0]
    # fp64 weight gradient of dy0 against relu(x sc + sh)
    xin = torch.relu(x.double() * xsc.double() + xsh.double()).reshape(n, h, w, ci).permute(0, 3, 1, 2)
    g = dy0.double().reshape(n, h, w, co).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xin.cpu(), (co, ci, 3, 3), g.cpu(), padding=1)
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())  # noqa: E731
    e0, e1 = rel(dw0.cpu(), ref), rel(dw1.cpu(), ref)
    print(f"wgrad rel err unfused {e0:.2e} fused {e1:.2e}")
    assert e1 < 2e-6 and e0 < 2e-6
    assert rel(dw1.cpu(), dw0.cpu().double()) < 2e-6


@pytest.mark.parametrize("form", ["pool", "pool_noskip", "heads1", "heads3"])
def test_sums_only_producers_record_max_da(form):
    """selunet_maxpool2_bwd / selunet_heads_bwd in sums-only mode with bnb.amax: the word is max |dA| of the
    dA the storing mode writes, bit for bit (the bound selunet_bn_bwd_stats_finalize_bound starts from)."""
    n, h, w, c = 2, 18, 36, 64
    m = n * h * w
    y = ((gen(m, c, seed=91) * 2).round() / 2).to(DEV)
    sc, sh, mean, invstd, _ = coefs(c, 92)
    res = []
    for fused in (False, True):
        rows = (K.query("selunet_maxpool2_bwd_slab_rows", n, h, w, c) if form.startswith("pool")
                else K.query("selunet_channel_slab_rows", m))
        bslab = torch.empty(rows, 3, c, device=DEV)
        word = torch.zeros(1, device=DEV)
        bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), K.ptr(bslab),
                           K.ptr(word) if fused else None)
        dz = None if fused else torch.empty(m, c, device=DEV)
        if form.startswith("pool"):
            dp = (gen(m // 4, c, seed=93) * 1e-2).to(DEV)
            ds = (gen(m, c, seed=94) * 1e-2).to(DEV) if form == "pool" else None
            K.call("selunet_maxpool2_bwd", K.ptr(y), n, h, w, c, K.ptr(sc), K.ptr(sh), K.ptr(dp), K.ptr(ds), K.ptr(dz),
                   bnb, K.F32, K.stream_ptr())
        else:
            nh = int(form[-1])
            wt = (gen(3, 64, seed=95) * 0.2).to(DEV).contiguous()
            g = [(gen(m, seed=96 + i) * 1e-3).to(DEV) for i in range(3)]
            slab = torch.empty(K.query("selunet_channel_slab_rows", m), nh * 65, device=DEV)
            K.call("selunet_heads_bwd", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(wt), nh,
                   *[K.ptr(g[i]) if i < nh else None for i in range(3)], K.ptr(dz), K.ptr(slab), bnb, K.F32,
                   K.stream_ptr())
        torch.cuda.synchronize()
        res.append((dz, word.item(), bslab.cpu()))
    (dz, _, b0), (_, wd, b1) = res
    assert torch.equal(b0, b1)
    assert wd == dz.abs().max().item() > 0


def _src_case(form, seed=100):
    """A 64-channel layer whose dA comes from a pool (with / without skip) or the heads: the BN state,
    the dA source for selunet_conv3x3_wgrad_x2_bn_src, and a call of the standalone apply it replaces."""
    n, h, w, c = 2, 20, 36, 64  # ragged 8x8 tiles in y
    m = n * h * w
    y = ((gen(m, c, seed=seed) * 2).round() / 2).to(DEV)  # coarse: ties inside the pool windows
    sc, sh, mean, invstd, coef = coefs(c, seed + 1)
    coef[0] = coef[0].abs() + 0.5
    keep = []
    if form.startswith("pool"):
        dp = (gen(m // 4, c, seed=seed + 2) * 1e-2).to(DEV)
        ds = (gen(m, c, seed=seed + 3) * 1e-2).to(DEV) if form == "pool" else None
        keep += [dp, ds]
        src = K.DaSource(K.DA_POOL, 0, K.ptr(dp), K.ptr(ds))

        def apply(dy, am):
            K.call("selunet_bn_bwd_apply_pool", K.ptr(y), n, h, w, c, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
                   K.ptr(coef), K.ptr(dp), K.ptr(ds), K.ptr(dy), K.ptr(am), K.F32, K.stream_ptr())
    else:
        nh = int(form[-1])
        wt = (gen(3, 64, seed=seed + 4) * 0.2).to(DEV).contiguous()
        g = [(gen(m, seed=seed + 5 + i) * 1e-3).to(DEV) for i in range(3)]
        gp = [K.ptr(g[i]) if i < nh else None for i in range(3)]
        keep += [wt, g]
        src = K.DaSource(K.DA_HEADS, nh, None, None, K.ptr(wt), (ctypes.c_void_p * 3)(*gp))

        def apply(dy, am):
            K.call("selunet_bn_bwd_apply_heads", K.ptr(y), m, K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd),
                   K.ptr(coef), K.ptr(wt), nh, *gp, K.ptr(dy), K.ptr(am), K.F32, K.stream_ptr())
    return (n, h, w, c), (y, sc, sh, mean, invstd, coef), src, apply, keep


@pytest.mark.parametrize("form", ["pool", "pool_noskip", "heads1", "heads3"])
def test_wgrad_x2_bn_src_equals_apply_then_wgrad(form):
    """selunet_conv3x3_wgrad_x2_bn_src with a pool / heads dA source (encoder_layer_1_2, decoder_layer_1_1)
    against selunet_bn_bwd_apply_pool / _heads + selunet_conv3x3_wgrad_x2: dy and max |dy| identical, the
    weight gradient within split-fp16 rounding of it and of the fp64 weight gradient."""
    (n, h, w, c), (y, sc, sh, mean, invstd, coef), src, apply, _keep = _src_case(form)
    m, ci = n * h * w, 64
    x = gen(m, ci, seed=171).to(DEV)
    xsc, xsh = (gen(ci, seed=172).abs() + 0.5).to(DEV), (gen(ci, seed=173) * 0.2).to(DEV)
    xw = (torch.relu(x * xsc + xsh)).abs().max().reshape(1).contiguous()
    gq = K.gather(n, h, w, 9, K.source(x, ci, xsc, xsh, relu=True, amax=xw))
    dy0 = torch.empty(m, c, device=DEV)
    am0 = torch.zeros(1, device=DEV)
    apply(dy0, am0)
    gp0 = K.gather(n, h, w, 1, K.source(dy0, c))
    wsb = K.query("selunet_conv3x3_wgrad_x2_ws_bytes", gp0, gq)
    ws = torch.empty(wsb // 4, device=DEV)
    dw0 = torch.empty(c, ci, 3, 3, device=DEV)
    K.call("selunet_conv3x3_wgrad_x2", gp0, gq, K.ptr(ws), wsb, K.ptr(dw0), K.ptr(am0), K.ptr(xw), None, K.stream_ptr())
    torch.cuda.synchronize()
    bound = (am0 * 37.0).contiguous()
    dy1 = torch.full((m, c), float("nan"), device=DEV)
    am1 = torch.zeros(1, device=DEV)
    dw1 = torch.empty(c, ci, 3, 3, device=DEV)
    gp1 = K.gather(n, h, w, 1, K.source(y, c))  # grid and channel count only
    bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), None)
    K.call("selunet_conv3x3_wgrad_x2_bn_src", gp1, gq, K.ptr(ws), wsb, K.ptr(dw1), K.ptr(bound), K.ptr(xw), None, bnb,
           K.ptr(coef), src, K.ptr(dy1), K.ptr(am1), K.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dy1.cpu(), dy0.cpu())
    assert am1.item() == am0.item()
    xin = torch.relu(x.double() * xsc.double() + xsh.double()).reshape(n, h, w, ci).permute(0, 3, 1, 2)
    g = dy0.double().reshape(n, h, w, c).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xin.cpu(), (c, ci, 3, 3), g.cpu(), padding=1)
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())  # noqa: E731
    e0, e1 = rel(dw0.cpu(), ref), rel(dw1.cpu(), ref)
    print(f"wgrad rel err unfused {e0:.2e} fused {e1:.2e}")
    assert e1 < 2e-6 and e0 < 2e-6
    assert rel(dw1.cpu(), dw0.cpu().double()) < 2e-6


def test_wgrad_x2_bn_src_argument_checks():
    (n, h, w, c), (y, sc, sh, mean, invstd, coef), src, _, _keep = _src_case("pool")
    x = gen(n * h * w, 128, seed=181).to(DEV)
    xw = x.abs().max().reshape(1).contiguous()
    gq = K.gather(n, h, w, 9, K.source(x, 128, amax=xw))
    y128 = torch.zeros(n * h * w, 128, device=DEV)
    ws = torch.empty(1 << 24, device=DEV)
    out = torch.empty(128, 128, 3, 3, device=DEV)
    bnb = K.BnBwdStats(K.ptr(y128), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), None)
    with pytest.raises(K.SelunetError):  # pool / heads sources are 64-channel forms
        K.call("selunet_conv3x3_wgrad_x2_bn_src", K.gather(n, h, w, 1, K.source(y128, 128)), gq, K.ptr(ws),
               ws.numel() * 4, K.ptr(out), K.ptr(xw), K.ptr(xw), None, bnb, K.ptr(coef), src, None, None,
               K.stream_ptr())
    bad = K.DaSource(7, 0, None, None)
    bnb = K.BnBwdStats(K.ptr(y), K.ptr(sc), K.ptr(sh), K.ptr(mean), K.ptr(invstd), None)
    with pytest.raises(K.SelunetError):
        K.call("selunet_conv3x3_wgrad_x2_bn_src", K.gather(n, h, w, 1, K.source(y, 64)), gq, K.ptr(ws), ws.numel() * 4,
               K.ptr(out), K.ptr(xw), K.ptr(xw), None, bnb, K.ptr(coef), bad, None, None, K.stream_ptr())


@pytest.mark.parametrize("n,size", [(4, 64), (2, 128)])
def test_step_fused_applies_on_off(monkeypatch, n, size):
    """Step-level check of the fused BN-backward applies: one fp32 training step with the
    applies fused into the split-fp16 weight gradients (SELUNET_FUSE_WGRAD_APPLY / _SRC = 1, default)
    against the same step with every apply standalone (= 0). The data gradients see bit-identical dy, so
    the loss and outputs are equal and every gradient agrees within split-fp16 rounding (the fused weight
    gradients split dy under the finalize's analytic |dy| bound instead of its exact max). At 64x64 the
    8x8 bottleneck layers run on the gather GEMM, whose epilogue must still write the max |dA| word the
    fused consumer's bound starts from — a missing word would leave k0 |dA| out of the bound."""
    import numpy as np
    from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch
    import selectivenet_for_semantic_segmentation_binary_amd as S
    from tests.test_gpu_model import build, train_step
    x, lab = make_batch(n, size, seed=4)
    xt, lt = torch.tensor(x, device=DEV), torch.tensor(lab, device=DEV)
    res = []
    for fused in ("1", "0"):
        monkeypatch.setenv("SELUNET_FUSE_WGRAD_APPLY", fused)
        monkeypatch.setenv("SELUNET_FUSE_WGRAD_SRC", fused)
        net = build(True)
        opt = S.Adam(net.parameters(), lr=1e-3)
        res.append([train_step(net, opt, xt, lt, True, 2) for _ in range(2)])
    (a0, a1), (b0, b1) = res
    assert a0["loss"] == b0["loss"] and np.array_equal(a0["output"], b0["output"])
    worst = 0.0
    for k in a0["grads"]:
        ga, gb = a0["grads"][k].astype(np.float64), b0["grads"][k].astype(np.float64)
        e = np.linalg.norm(ga - gb) / max(np.linalg.norm(gb), 1e-30)
        worst = max(worst, e)
        assert e <= 1e-5, (k, e)
    assert abs(a1["loss"] - b1["loss"]) <= 1e-5 * abs(b1["loss"]), (a1["loss"], b1["loss"])
    print(f"fused vs unfused applies at {n}x{size}^2: worst gradient rel L2 {worst:.2e}")
