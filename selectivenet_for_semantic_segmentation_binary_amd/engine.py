"""Kernel sequencing for one UNet_B forward / backward on the MI355X (no autograd inside).

This is the host side of the hot path: it mirrors `UNet_B.forward` (model.py:68-103) layer by
layer, but every op is a call into libselunet.so. Layout in HBM: activations NHWC, element
type `dt` (fp32 for the parity configuration, bf16 for the fast one); per-layer state kept for
the backward is only the pre-BN conv output `y` (its BN+ReLU is re-applied by whichever kernel
reads it), the folded BN scale/shift/mean/invstd, the 3 pooled tensors and the 3 up-sampled
tensors — `torch.cat` is never materialised (the decoder GEMMs read two sources).

Backward order (train.py:208 autograd, restated explicitly):
heads -> dec1_1 -> dec1_2 (dgrad split into d(up1), d(skip1)) -> unpool1 -> dec2_1 -> ... ->
bottleneck -> pool3 backward (+ d(skip3)) -> enc3_2 -> ... -> enc1_1 (no data gradient).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from collections import OrderedDict
from dataclasses import dataclass, field

import torch

from . import _lib as K
from . import layout as LY

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
# fp32 BatchNorm statistics: channel groups with mean^2 > BN_CENTER_RATIO x the one-pass variance get
# the centered second pass over y (selunet_bn_centered_partials_adaptive); None: every channel does
# (SELUNET_BN_FLAG_RATIO: the threshold for A/B runs)
BN_CENTER_RATIO = (None if os.environ.get("SELUNET_BN_TWOPASS", "0") == "1"
                   else float(os.environ.get("SELUNET_BN_FLAG_RATIO", "1.0")))
FIRST_KPAD = 32  # packed K of encoder_layer_1_1 (9 * C_in <= 27), see selunet_first_conv_fwd


# split-fp16 ("x2") kernel form of a 3x3 layer (selunet_conv3x3_x2; a split-fp16 Winograd F(2,3) form was
# built in round 4 and retired in round 6: slower on every layer)
X2_MODES = ("x2",)


def _rup(a, b):
    return (a + b - 1) // b * b


def fp32_conv_path() -> str:
    """Which kernels an fp32 training step runs its convolutions on in this process (SELUNET_X2,
    SELUNET_WINO): "split-fp16" (the default) or "exact-fp32 (Winograd|direct)"."""
    if os.environ.get("SELUNET_X2", "1") != "0":
        return "split-fp16"
    return "exact-fp32 (" + ("direct" if os.environ.get("SELUNET_WINO", "1") == "0" else "Winograd") + ")"


@dataclass
class BNState:
    y: torch.Tensor          # pre-BN conv output (no bias), NHWC [M][C]
    mean: torch.Tensor
    invstd: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor
    n: int
    h: int
    w: int
    c: int
    amax: torch.Tensor = None  # range word of relu(bn(y)) (split-fp16 layers, selunet_act_bound)
    name: str = ""

    def src(self):
        return K.source(self.y, self.c, self.scale, self.shift, relu=True, amax=self.amax)


@dataclass
class WPack:
    """A conv layer's weight operands for the step: fwd / dgrad packs, the forward's K, output
    channels, and the kernel form: "direct" (halo / gather GEMM in the compute dtype), "wino" (fp32
    Winograd F(2,3)) or "x2" (fp32 on split-fp16 operands, selunet_conv3x3_x2)."""
    fwd: torch.Tensor
    dgrad: torch.Tensor
    kpad: int
    co: int
    mode: str = "direct"


@dataclass
class DGrad:
    """A data gradient plus the per-workgroup partial sums its producing kernel wrote alongside:
    BN-backward sums [rows][3][C] for a CBR block's dA, or column sums [rows][C] for the up-sampled
    half of a torch.cat gradient (the ConvTranspose2d bias gradient). `apply` (optional) replaces dA for
    a producer that ran in sums-only mode (t is None): apply(dy, coef, amax_word_or_None) enqueues the
    BN-backward apply that forms dA on the fly (selunet_bn_bwd_apply_heads / _pool)."""
    t: torch.Tensor
    slab: torch.Tensor = None
    rows: int = 0
    apply: object = None
    da_word: bool = False  # the producer recorded max |t| in ctx.words["da:" + layer] (fused apply's bound)
    src: object = None  # K.DaSource: dA of a sums-only producer (pool / heads) the fused weight gradient forms


def bnb_for(st: BNState, slab, amax=None) -> K.BnBwdStats:
    """amax (nullable): the word a sums-only pool / heads producer records max |dA| into."""
    return K.BnBwdStats(K.ptr(st.y), K.ptr(st.scale), K.ptr(st.shift), K.ptr(st.mean), K.ptr(st.invstd), K.ptr(slab),
                        K.ptr(amax))


@dataclass
class Ctx:
    dt: torch.dtype
    training: bool
    selective: bool
    shape: tuple
    x: torch.Tensor = None
    entry: object = None     # the launch-plan cache entry this context belongs to (None: uncached)
    bn: dict = field(default_factory=dict)
    pools: dict = field(default_factory=dict)
    ups: dict = field(default_factory=dict)
    wpack: dict = field(default_factory=dict)
    words: dict = field(default_factory=dict)  # operand range words (split-fp16 layers) by key
    x2: bool = False                           # some layer of this pass runs split-fp16


class _Entry:
    """One recorded forward (and its backward plans) with the activations it owns."""

    def __init__(self, key):
        self.key = key
        self.plan = None
        self.ctx = None
        self.bwd = {}
        self.busy = False


class Engine:
    """Sequencer; parameters/buffers are passed in as dicts of tensors.

    Launch plans: the first forward (and backward) for a given input shape / mode / parameter set
    runs the Python sequencing below while recording every C-ABI call (`_lib.Plan`); later calls
    with the same signature replay the recorded launches with the per-call buffers (input, head
    outputs, head gradients, gradient buffer) rebound, so the host cost of a training step is the
    ctypes calls alone — what keeps small per-GPU batches (8-GPU strong scaling) GPU-bound. The
    activations a plan owns stay allocated between steps (the caching allocator would have held
    them anyway); a forward whose backward is pending keeps its plan busy, and a second forward of
    the same shape then records (or, past MAX_PLANS, runs unrecorded). SELUNET_NO_PLANS=1 disables
    plans."""

    MAX_PLANS = 4  # per signature

    def __init__(self, dt: torch.dtype = torch.float32):
        self.dt = dt
        self.code = K.dtype_code(dt)
        self.bke = 128 // torch.empty((), dtype=dt).element_size()
        self.plans_enabled = os.environ.get("SELUNET_NO_PLANS", "0") != "1"
        self.deterministic = os.environ.get("SELUNET_DETERMINISTIC", "1") != "0"
        # fp32 training: 3x3 layers on split-fp16 operands (selunet_conv3x3_x2); SELUNET_X2=0 keeps
        # the exact-fp32-MFMA kernels (Winograd / direct)
        self.x2 = dt == torch.float32 and os.environ.get("SELUNET_X2", "1") != "0"
        # fp32 training BN statistics: the conv epilogue sums y - c with c = the previous step's batch
        # mean (selunet_epilogue.stats_center), so the one-pass variance is exact enough for almost
        # every channel after the first step and the centered pass re-reads (almost) nothing;
        # SELUNET_BN_SHIFT=0 keeps c = 0
        self.bn_shift = dt == torch.float32 and BN_CENTER_RATIO is not None and \
            os.environ.get("SELUNET_BN_SHIFT", "1") != "0"
        # split-fp16 training: the BN-backward apply of layers whose dA is stored runs inside their weight
        # gradient (selunet_conv3x3_wgrad_x2_bn); SELUNET_FUSE_WGRAD_APPLY=0 keeps the separate apply
        self.fuse_wgrad_apply = os.environ.get("SELUNET_FUSE_WGRAD_APPLY", "1") != "0"
        # ... and for the 64-channel layers whose dA is formed on the fly (encoder_layer_1_2 from the pool's
        # gradient, decoder_layer_1_1 from the heads'): SELUNET_FUSE_WGRAD_SRC=0 keeps their separate applies
        self.fuse_wgrad_src = os.environ.get("SELUNET_FUSE_WGRAD_SRC", "1") != "0"
        self._plans = OrderedDict()  # signature -> [_Entry]

    # ------------------------------------------------------------------ small helpers
    def _reduce(self, slab, rows, cols, out64=None, out32=None):
        ws = K.keep(torch.empty(K.query("selunet_reduce_ws_bytes", cols) // 8, dtype=torch.float64, device=slab.device))
        K.call("selunet_reduce_rows", K.ptr(slab), rows, cols, K.ptr(ws), K.ptr(out64), K.ptr(out32), self.stream)

    @property
    def stream(self):
        return K.stream_ptr()

    def _wgrad(self, gp, gq, packed):
        """packed = P^T Q (weight gradient, fp32 [ni][ld]), overwritten. bf16 (default): the pixel
        splits write partials to a workspace reduced in a fixed order — bit-reproducible, and at
        small per-GPU batches faster than the fp32 atomics it replaces (~150 MB of atomic adds per
        3x3 layer, independent of the batch): +8% images/s at 16 images per GPU, equal at 128.
        SELUNET_DETERMINISTIC=0 selects zero + atomics."""
        if not self.deterministic:
            K.call("selunet_memset", K.ptr(packed), 0, packed.numel() * 4, self.stream)
            K.call("selunet_gemm_wgrad", gp, gq, K.ptr(packed), self.code, self.stream)
            return
        wsb = K.query("selunet_gemm_wgrad_ws_bytes", gp, gq, self.code)
        if wsb < 0:
            raise RuntimeError(f"selunet_gemm_wgrad_ws_bytes: {K.load().selunet_last_error().decode()}")
        ws = K.keep(torch.empty(max(wsb // 4, 1), dtype=torch.float32, device=packed.device)) if wsb > 0 else None
        K.call("selunet_gemm_wgrad_ws", gp, gq, K.ptr(packed), K.ptr(ws), wsb, self.code, self.stream)

    def _wgrad_x2(self, gp, gq, dyw, srcs, out):
        """3x3 weight gradient on split-fp16 operands (selunet_conv3x3_wgrad_x2) when dY and every
        input source carry range words and the shapes fit; False: not taken."""
        words = [sr.amax for sr in srcs]
        if dyw is None or any(wd is None for wd in words):
            return False
        wsb = K.query("selunet_conv3x3_wgrad_x2_ws_bytes", gp, gq)
        if wsb <= 0:
            return False
        ws = K.keep(torch.empty(wsb // 4, dtype=torch.float32, device=out.device))
        K.call("selunet_conv3x3_wgrad_x2", gp, gq, K.ptr(ws), wsb, K.ptr(out), K.ptr(dyw), K.ptr(words[0]),
               K.ptr(words[1]) if len(words) > 1 else None, self.stream)
        return True

    def _wgrad_param(self, gp, gq, layout, ni, ld, out):
        """Weight gradient straight into the parameter's gradient in the reference layout
        (layout WG_CONV3X3: [co][ci][3][3], WG_CONVT: [ci][co][2][2]); deterministic bf16 path: the
        split reduction writes that layout itself (no packed copy, no unpack launch)."""
        dev = out.device
        if self.deterministic:
            wsb = K.query("selunet_gemm_wgrad_ws_bytes", gp, gq, self.code)
            if wsb < 0:
                raise RuntimeError(f"selunet_gemm_wgrad_ws_bytes: {K.load().selunet_last_error().decode()}")
            if wsb > 0:
                ws = K.keep(torch.empty(wsb // 4, dtype=torch.float32, device=dev))
                K.call("selunet_gemm_wgrad_ws_to", gp, gq, None, K.ptr(ws), wsb, layout, K.ptr(out), self.code,
                       self.stream)
                return
        packed = K.keep(torch.empty(ni, ld, dtype=torch.float32, device=dev))
        self._wgrad(gp, gq, packed)
        if layout == K.WG_CONV3X3:
            K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), ni, out.shape[1], ld, K.ptr(out),
                   self.stream)
        else:
            K.call("selunet_unpack_convT_grad", K.ptr(packed), ni, out.shape[1], K.ptr(out), self.stream)

    @staticmethod
    def _layer_hw(name, hw):
        f = 1 << (int(name.split("_")[2]) - 1)  # encoder/decoder level k runs at 1 / 2^(k-1)
        return hw[0] // f, hw[1] // f

    @staticmethod
    def _concat_c0(name, ci):
        concat = name.startswith("decoder_layer") and name.endswith("_2") and name != "decoder_layer_4_2"
        return ci // 2 if concat else ci  # torch.cat((unpool, skip)) inputs: two equal sources

    def _shape_ok(self, query, name, ci, co, hw, need_dgrad):
        h, w = self._layer_hw(name, hw)
        ok = K.query(query, h, w, ci, self._concat_c0(name, ci), co) == 1
        return ok and (not need_dgrad or K.query(query, h, w, co, co, ci) == 1)

    def _wino_ok(self, name, ci, co, hw, need_dgrad):
        """fp32 layers whose forward (and data gradient) run as the Winograd F(2,3) kernel
        (selunet_conv3x3_wino): decided from the layer's resolution and channels."""
        if self.dt != torch.float32 or hw is None or name == "encoder_layer_1_1":
            return False
        return self._shape_ok("selunet_conv3x3_wino_ok", name, ci, co, hw, need_dgrad)

    def _x2_ok(self, name, ci, co, hw, need_dgrad, training):
        """fp32 training layers on split-fp16 operands (selunet_conv3x3_x2). Training only: the range
        word of a BN+ReLU input (selunet_act_bound) holds for batch statistics."""
        if not (self.x2 and training) or hw is None or name == "encoder_layer_1_1":
            return False
        return self._shape_ok("selunet_conv3x3_x2_ok", name, ci, co, hw, need_dgrad)

    def pack_weights(self, P, need_dgrad=True, hw=None, training=False, heads=()):
        """fp32 master weights -> GEMM operand layouts in the compute dtype (one launch for all);
        fp32 layers at input resolution hw get the split-fp16 (training) or Winograd operands.
        heads: (name, channels) of the output heads whose weights / biases are gathered, in the same
        launch, into the contiguous fp32 operands of the heads kernel (packs["heads"] = (w, b)).
        Returns name -> WPack."""
        dev = P["encoder_layer_1_2.0.weight"].device
        packs = {}
        pl = K.PackList()
        for name, ci, co in LY.CBR_LAYERS:
            w = P[f"{name}.0.weight"]
            ci = w.shape[1]
            dg = None
            if self._x2_ok(name, ci, co, hw, need_dgrad, training):
                mode, kpad, kind = "x2", 9 * ci, K.PACK_CONV3X3_X2
                fwd = K.keep(torch.empty(co * kpad + co, dtype=torch.float32, device=dev))
                if need_dgrad:
                    dg = K.keep(torch.empty(ci * (kpad // ci) * co + ci, dtype=torch.float32, device=dev))
            else:
                if self._wino_ok(name, ci, co, hw, need_dgrad):
                    mode, kpad, taps, kind = "wino", 12 * ci, 12, K.PACK_CONV3X3_WINO
                else:
                    kpad = FIRST_KPAD if name == "encoder_layer_1_1" else _rup(9 * ci, self.bke)
                    mode, taps, kind = "direct", 9, K.PACK_CONV3X3
                fwd = K.keep(torch.empty(co, kpad, dtype=self.dt, device=dev))
                if need_dgrad and name != "encoder_layer_1_1":
                    dg = K.keep(torch.empty(ci, taps * co, dtype=self.dt, device=dev))
            pl.d[pl.n] = K.PackDesc(K.ptr(w), K.ptr(fwd), K.ptr(dg), kind, co, ci, kpad, 0)
            pl.n += 1
            packs[name] = WPack(fwd, dg, kpad, co, mode)
        x2 = any(wp.mode in X2_MODES for wp in packs.values())
        for name, ci, co in LY.UNPOOLS:
            w = P[f"{name}.weight"]
            if x2:  # ConvTranspose2d forward / data gradient on split-fp16 operands (selunet_gemm_gather_x2)
                fwd = K.keep(torch.empty(4 * co * ci + 4 * co, dtype=torch.float32, device=dev))
                dg = K.keep(torch.empty(ci * 4 * co + ci, dtype=torch.float32, device=dev)) if need_dgrad else None
                pl.d[pl.n] = K.PackDesc(K.ptr(w), K.ptr(fwd), K.ptr(dg), K.PACK_CONVT_X2, co, ci, ci, 0)
            else:
                fwd = K.keep(torch.empty(4 * co, ci, dtype=self.dt, device=dev))
                dg = K.keep(torch.empty(ci, 4 * co, dtype=self.dt, device=dev)) if need_dgrad else None
                pl.d[pl.n] = K.PackDesc(K.ptr(w), K.ptr(fwd), K.ptr(dg), K.PACK_CONVT, co, ci, 0, 0)
            pl.n += 1
            packs[name] = WPack(fwd, dg, ci, co, "x2" if x2 else "direct")
        if heads:
            no = sum(c for _, c in heads)
            hw_, hb_ = (K.keep(torch.empty(no, k, dtype=torch.float32, device=dev)) for k in (64, 1))
            k = 0
            if pl.n + 2 * len(heads) > K.PACK_MAX:
                raise ValueError(f"{len(heads)} heads: more weight-pack entries than SELUNET_PACK_MAX")
            for h, c in heads:
                for t, dst, n in ((P[f"{h}.weight"], hw_[k:], c * 64), (P[f"{h}.bias"], hb_[k:], c)):
                    pl.d[pl.n] = K.PackDesc(K.ptr(t), K.ptr(dst), None, K.PACK_COPY, n, 1, 0, 0)
                    pl.n += 1
                k += c
            packs["heads"] = (hw_, hb_.view(no))
        K.call("selunet_pack_weights", pl, self.code, self.stream)
        return packs

    def _word(self, ctx, key):
        """The range word `key` of this forward/backward (zeroed at the start of the forward)."""
        return ctx.words[key]

    # ------------------------------------------------------------------ forward pieces
    def _conv3x3(self, g, b, n_cols, kpad, ep, mode, srcs=()):
        """A 3x3 conv (forward or data gradient) through the direct halo / gather kernels, or the
        fp32 Winograd / split-fp16 kernel when the layer's operands were packed for it (srcs: the
        gather's sources, whose range words the split-fp16 kernel reads)."""
        if mode in X2_MODES:
            words = [s.amax for s in srcs]
            if any(wd is None for wd in words):
                raise RuntimeError("split-fp16 conv: a source without its range word")
            K.call("selunet_conv3x3_x2", g, K.ptr(b), n_cols, ep,
                   K.ptr(words[0]), K.ptr(words[1]) if len(words) > 1 else None, self.stream)
        elif mode == "wino":
            K.call("selunet_conv3x3_wino", g, K.ptr(b), n_cols, ep, self.stream)
        else:
            K.call("selunet_gemm_gather", g, K.ptr(b), n_cols, kpad, ep, self.code, self.stream)

    def _cbr(self, ctx, name, P, B, n, h, w, *srcs, taps=9, first_x=None):
        """CBR_2D forward (model.py:9-15): conv (+ BN batch statistics in its epilogue), BN finalize.
        first_x: the network input (NCHW fp32) for encoder_layer_1_1, convolved directly."""
        wp = ctx.wpack[name]
        fwd, kpad, co = wp.fwd, wp.kpad, wp.co
        M = n * h * w
        dev = fwd.device
        y = K.keep(torch.empty(M, co, dtype=self.dt, device=dev))
        stats = None
        if first_x is not None:
            rows = K.query("selunet_first_conv_rows", n, h, w)
        else:
            g = K.gather(n, h, w, taps, *srcs)
            rows = (K.query("selunet_conv3x3_x2_stats_rows", g, co) if wp.mode in X2_MODES
                    else K.query("selunet_gemm_stats_rows", g, co, self.code))
        center = None
        if ctx.training:
            stats = K.keep(torch.empty(rows, 2, co, dtype=torch.float32, device=dev))
            if self.bn_shift:  # (zero when recorded; a replayed step finds the previous step's mean here)
                center = K.keep(torch.zeros(co, dtype=torch.float32, device=dev))
        if first_x is not None:
            K.call("selunet_first_conv_fwd_centered", K.ptr(first_x), n, first_x.shape[1], h, w, K.ptr(fwd),
                   K.ptr(y), K.ptr(stats), K.ptr(center), self.code, self.stream)
        else:
            ep = K.Epilogue(K.ptr(y), None, None, K.ptr(stats), K.EP_PLAIN, 0)
            ep.stats_center = K.ptr(center)
            self._conv3x3(g, fwd, co, kpad, ep, wp.mode, srcs)
        mean, invstd, scale, shift = (K.keep(torch.empty(co, dtype=torch.float32, device=dev)) for _ in range(4))
        if ctx.training and self.dt == torch.float32:
            # fp32 (parity): two-pass statistics — the epilogue's sums give the batch mean, a second
            # pass over y sums (y - mean) and (y - mean)^2 for the variance, then the finalize with the
            # running-statistic updates (selunet_bn_centered_partials)
            # (adaptive: only channel groups whose mean^2 exceeds BN_CENTER_RATIO x the one-pass variance
            # are re-read — where E[y^2] - mean^2 loses digits; SELUNET_BN_TWOPASS=1 re-reads all)
            ws = K.keep(torch.empty(K.query("selunet_reduce_ws_bytes", 2 * co) // 8, dtype=torch.float64, device=dev))
            uvar = K.keep(torch.zeros(co, dtype=torch.float32, device=dev)) if BN_CENTER_RATIO is not None else None
            if center is not None:  # shifted sums: mean, the one-pass variance or -1 where it is not exact enough
                K.call("selunet_bn_stats_finalize_shifted", K.ptr(stats), rows, K.ptr(ws), M, co, K.ptr(center),
                       K.ptr(P[f"{name}.0.bias"]), K.ptr(P[f"{name}.1.weight"]), K.ptr(P[f"{name}.1.bias"]),
                       BN_CENTER_RATIO, K.ptr(mean), K.ptr(uvar), K.ptr(invstd), K.ptr(scale), K.ptr(shift),
                       self.stream)
            else:
                K.call("selunet_bn_stats_finalize", K.ptr(stats), rows, K.ptr(ws), None, M, co,
                       K.ptr(P[f"{name}.0.bias"]), K.ptr(P[f"{name}.1.weight"]), K.ptr(P[f"{name}.1.bias"]),
                       None, K.ptr(uvar), None, 1.0 if uvar is not None else BN_MOMENTUM, BN_EPS, K.ptr(mean),
                       K.ptr(invstd), K.ptr(scale), K.ptr(shift), self.stream)
            rows2 = K.query("selunet_bn_centered_rows", M)
            slab2 = K.keep(torch.empty(rows2, 2, co, dtype=torch.float32, device=dev))
            if uvar is not None:  # (shifted: the flags decide, ratio +inf)
                K.call("selunet_bn_centered_partials_adaptive", K.ptr(y), M, co, K.ptr(mean), K.ptr(uvar),
                       float("inf") if center is not None else BN_CENTER_RATIO, K.ptr(slab2), self.code,
                       self.stream)
            else:
                K.call("selunet_bn_centered_partials", K.ptr(y), M, co, K.ptr(mean), K.ptr(slab2), self.code,
                       self.stream)
            # (+ the split-fp16 range word of relu(bn(y)) in the same launch, see below)
            bound = self._word(ctx, "act:" + name) if ctx.x2 else None
            K.call("selunet_bn_stats_finalize_centered_bound", K.ptr(slab2), rows2, K.ptr(ws), None, M, co,
                   K.ptr(mean), K.ptr(P[f"{name}.0.bias"]), K.ptr(P[f"{name}.1.weight"]), K.ptr(P[f"{name}.1.bias"]),
                   K.ptr(B[f"{name}.1.running_mean"]), K.ptr(B[f"{name}.1.running_var"]),
                   K.ptr(B[f"{name}.1.num_batches_tracked"]), BN_MOMENTUM, BN_EPS,
                   K.ptr(mean), K.ptr(invstd), K.ptr(scale), K.ptr(shift), K.ptr(bound), self.stream)
        elif ctx.training:  # statistics slab -> fp64 column sums -> batch mean/invstd, running stats: one launch
            ws = K.keep(torch.empty(K.query("selunet_reduce_ws_bytes", 2 * co) // 8, dtype=torch.float64, device=dev))
            K.call("selunet_bn_stats_finalize", K.ptr(stats), rows, K.ptr(ws), None, M, co,
                   K.ptr(P[f"{name}.0.bias"]), K.ptr(P[f"{name}.1.weight"]), K.ptr(P[f"{name}.1.bias"]),
                   K.ptr(B[f"{name}.1.running_mean"]), K.ptr(B[f"{name}.1.running_var"]),
                   K.ptr(B[f"{name}.1.num_batches_tracked"]), BN_MOMENTUM, BN_EPS,
                   K.ptr(mean), K.ptr(invstd), K.ptr(scale), K.ptr(shift), self.stream)
        else:
            K.call("selunet_bn_finalize", None, M, co, K.ptr(P[f"{name}.0.bias"]), K.ptr(P[f"{name}.1.weight"]),
                   K.ptr(P[f"{name}.1.bias"]), K.ptr(B[f"{name}.1.running_mean"]), K.ptr(B[f"{name}.1.running_var"]),
                   K.ptr(B[f"{name}.1.num_batches_tracked"]), BN_MOMENTUM, BN_EPS, 0,
                   K.ptr(mean), K.ptr(invstd), K.ptr(scale), K.ptr(shift), self.stream)
        st = BNState(y, mean, invstd, scale, shift, n, h, w, co, name=name)
        # range word of relu(bn(y)) for the split-fp16 consumers. The Samuelson bound |xhat| <= sqrt(M - 1)
        # holds for statistics over THIS rank's M values (per-rank BatchNorm, DataParallel replica
        # semantics); a synchronized BatchNorm would need M = the global count here.
        # (fp32 training folds it into the centered finalize: max_c |gamma_c| sqrt(M) + |beta_c|)
        if ctx.x2:
            st.amax = self._word(ctx, "act:" + name)
            if not (ctx.training and self.dt == torch.float32):
                K.call("selunet_act_bound", K.ptr(P[f"{name}.1.weight"]), K.ptr(P[f"{name}.1.bias"]), co, M,
                       K.ptr(st.amax), self.stream)
        ctx.bn[name] = st
        return st

    def _pool(self, ctx, key, st: BNState):
        out = K.keep(torch.empty(st.n * (st.h // 2) * (st.w // 2), st.c, dtype=self.dt, device=st.y.device))
        K.call("selunet_maxpool2_fwd", K.ptr(st.y), st.n, st.h, st.w, st.c, K.ptr(st.scale), K.ptr(st.shift),
               K.ptr(out), self.code, self.stream)
        ctx.pools[key] = out
        return out

    def _up(self, ctx, name, P, st: BNState):
        wp = ctx.wpack[name]
        fwd, ci, co = wp.fwd, wp.kpad, wp.co
        out = K.keep(torch.empty(st.n * 2 * st.h * 2 * st.w, co, dtype=self.dt, device=st.y.device))
        g = K.gather(st.n, st.h, st.w, 1, st.src())
        ep = K.Epilogue(K.ptr(out), None, K.ptr(P[f"{name}.bias"]), None, K.EP_SCATTER2X, 0)
        if ctx.x2:  # range word of the up-sampled tensor (exact max, the epilogue's atomic)
            ep.amax = K.ptr(self._word(ctx, "up:" + name))
        if wp.mode == "x2":
            K.call("selunet_gemm_gather_x2", g, K.ptr(fwd), 4 * co, ci, ep, K.ptr(st.amax), None, self.stream)
        else:
            K.call("selunet_gemm_gather", g, K.ptr(fwd), 4 * co, ci, ep, self.code, self.stream)
        ctx.ups[name] = out
        return out

    # ------------------------------------------------------------------ plan cache
    def _signature(self, x, P, B, selective, training, need_backward):
        return (tuple(x.shape), x.device.index, bool(selective), bool(training), bool(need_backward), self.stream,
                tuple(t.data_ptr() for t in P.values()), tuple(t.data_ptr() for t in B.values()))

    def _entry_for(self, sig):
        lst = self._plans.get(sig)
        if lst is None:
            lst = self._plans[sig] = []
            while len(self._plans) > 2 * self.MAX_PLANS:  # evict the oldest signature with no busy entry
                for k, v in self._plans.items():
                    if k != sig and not any(e.busy for e in v):
                        del self._plans[k]
                        break
                else:
                    break
        self._plans.move_to_end(sig)
        for e in lst:
            if not e.busy:
                return e
        if len(lst) < self.MAX_PLANS:
            e = _Entry(sig)
            lst.append(e)
            return e
        return None

    @staticmethod
    def release(ctx):
        """Mark the plan of a forward whose backward will not run (autograd graph freed) reusable."""
        if ctx is not None and ctx.entry is not None:
            ctx.entry.busy = False

    def forward(self, x, P, B, selective, training, need_backward=False, ce_heads=None):
        """x: [N, Cin, H, W] fp32 contiguous. Returns (heads tuple, ctx); the heads are new tensors:
        [N, H, W] logits for UNet_B, or, with ce_heads = [(head, channels)] (the CE `UNet`),
        NCHW [N, channels, H, W] logits per head."""
        assert x.dim() == 4 and x.is_contiguous() and x.dtype == torch.float32
        n, cin, H, W = x.shape
        if H % 8 or W % 8:
            raise ValueError(f"UNet_B needs H and W divisible by 8 (three 2x2 poolings); got {H}x{W}")
        if ce_heads is None:
            nheads = 3 if selective else 1
            outs = tuple(torch.empty(n, H, W, dtype=torch.float32, device=x.device) for _ in range(nheads))
        else:
            ce_heads = tuple(ce_heads)
            outs = tuple(torch.empty(n, c, H, W, dtype=torch.float32, device=x.device) for _, c in ce_heads)
        e = self._entry_for(self._signature(x, P, B, selective, training, need_backward) + (ce_heads,)) \
            if self.plans_enabled else None
        slots = {"x": x, **{f"out{i}": o for i, o in enumerate(outs)}}
        if e is None:
            ctx = self._forward_impl(x, P, B, selective, training, need_backward, outs, ce_heads)
        elif e.plan is not None:
            e.plan.replay(slots)
            ctx = e.ctx
            ctx.x = x
        else:
            plan = K.Plan(slots)
            with K.recording(plan):
                ctx = self._forward_impl(x, P, B, selective, training, need_backward, outs, ce_heads)
            e.plan, e.ctx = plan, ctx
            ctx.entry = e
        if e is not None and training and need_backward:
            e.busy = True
        return outs, ctx

    def _forward_impl(self, x, P, B, selective, training, need_backward, outs, ce_heads=None):
        n, cin, H, W = x.shape
        ctx = Ctx(self.dt, training, selective, (n, cin, H, W), x=x)
        ctx.ce_heads = ce_heads
        heads = LY.HEADS if selective else LY.HEADS[:1]
        heads = list(ce_heads) if ce_heads is not None else [(h, 1) for h in heads]
        if sum(c for _, c in heads) > 8:
            raise ValueError(f"the heads have {sum(c for _, c in heads)} output channels; the MI355X heads kernel "
                             "takes at most 8")
        ctx.wpack = self.pack_weights(P, need_dgrad=training and need_backward, hw=(H, W), training=training,
                                      heads=heads)
        hw, hb = ctx.wpack.pop("heads")
        ctx.x2 = any(wp.mode in X2_MODES for wp in ctx.wpack.values())
        if ctx.x2:  # the operand range words of this step, zeroed for their atomic-max producers
            # act: relu(bn(y)); dy / du: conv-output and up-sampled gradients; da: the exact max |dA| its
            # producer stores; dyb: the bound of |dy| selunet_bn_bwd_stats_finalize_bound derives from it
            keys = [f"{k}:{nm}" for nm, _, _ in LY.CBR_LAYERS for k in ("act", "dy", "du", "da", "dyb")]
            keys += ["up:" + nm for nm, _, _ in LY.UNPOOLS]
            buf = K.keep(torch.empty(len(keys), dtype=torch.float32, device=x.device))
            K.call("selunet_memset", K.ptr(buf), 0, buf.numel() * 4, self.stream)
            ctx.words = {k: buf[i:i + 1] for i, k in enumerate(keys)}
        c = lambda name, h, w, *s: self._cbr(ctx, name, P, B, n, h, w, *s)  # noqa: E731
        h1, w1, h2, w2, h3, w3, h4, w4 = H, W, H // 2, W // 2, H // 4, W // 4, H // 8, W // 8
        # first layer (C_in = 3 or 2): convolved straight from the NCHW fp32 input
        e11 = self._cbr(ctx, "encoder_layer_1_1", P, B, n, h1, w1, first_x=x)
        e12 = c("encoder_layer_1_2", h1, w1, e11.src())
        p1 = self._pool(ctx, "pool1", e12)
        wd = lambda st: st.amax  # noqa: E731  a pooled copy keeps its source's range
        e21 = c("encoder_layer_2_1", h2, w2, K.source(p1, 64, amax=wd(e12)))
        e22 = c("encoder_layer_2_2", h2, w2, e21.src())
        p2 = self._pool(ctx, "pool2", e22)
        e31 = c("encoder_layer_3_1", h3, w3, K.source(p2, 128, amax=wd(e22)))
        e32 = c("encoder_layer_3_2", h3, w3, e31.src())
        p3 = self._pool(ctx, "pool3", e32)
        b42 = c("decoder_layer_4_2", h4, w4, K.source(p3, 256, amax=wd(e32)))
        b41 = c("decoder_layer_4_1", h4, w4, b42.src())
        u3 = self._up(ctx, "unpool3", P, b41)
        uw = lambda nm: ctx.words.get("up:" + nm)  # noqa: E731
        d32 = c("decoder_layer_3_2", h3, w3, K.source(u3, 256, amax=uw("unpool3")), e32.src())
        d31 = c("decoder_layer_3_1", h3, w3, d32.src())
        u2 = self._up(ctx, "unpool2", P, d31)
        d22 = c("decoder_layer_2_2", h2, w2, K.source(u2, 128, amax=uw("unpool2")), e22.src())
        d21 = c("decoder_layer_2_1", h2, w2, d22.src())
        u1 = self._up(ctx, "unpool1", P, d21)
        d12 = c("decoder_layer_1_2", h1, w1, K.source(u1, 64, amax=uw("unpool1")), e12.src())
        d11 = c("decoder_layer_1_1", h1, w1, d12.src())
        M = n * H * W
        if ce_heads is not None:
            return self._heads_fwd_planes(ctx, d11, outs, ce_heads, n, H * W, hw, hb)
        o = list(outs) + [None] * (3 - len(outs))
        K.call("selunet_heads_fwd", K.ptr(d11.y), M, K.ptr(d11.scale), K.ptr(d11.shift), K.ptr(hw), K.ptr(hb),
               len(heads), K.ptr(o[0]), K.ptr(o[1]), K.ptr(o[2]), self.code, self.stream)
        ctx.head_w = hw
        return ctx

    # ------------------------------------------------------------------ N-output heads (CE UNet)
    @staticmethod
    def _planes(tensors, ce_heads, hw, with_slab=False):
        """selunet_head_planes over per-head NCHW tensors [N, c, H, W]; with_slab: the slab offsets of
        each output's weight (64) and bias sums in the heads' segment of the gradient buffer
        (registration order: weight [c, 64] then bias [c] per head)."""
        d = K.HeadPlanes()
        k, off = 0, 0
        for t, (_, c) in zip(tensors, ce_heads):
            for j in range(c):
                d.plane[k] = t.data_ptr() + j * hw * 4
                d.img_stride[k] = c * hw
                d.w_off[k] = off + j * 64
                d.b_off[k] = off + c * 64 + j
                k += 1
            off += c * 65
        d.n, d.hw, d.row_len = k, hw, off
        return d

    def _heads_fwd_planes(self, ctx, d11, outs, ce_heads, n, hw, w, b):
        """w [no][64], b [no]: the heads' current weights (gathered by pack_weights)."""
        K.call("selunet_heads_fwd_planes", K.ptr(d11.y), n * hw, K.ptr(d11.scale), K.ptr(d11.shift), K.ptr(w), K.ptr(b),
               self._planes(outs, ce_heads, hw), self.code, self.stream)
        ctx.head_w = w
        return ctx

    # ------------------------------------------------------------------ backward pieces
    def _cbr_bwd(self, ctx, name, dg: DGrad, G, input_srcs, dgrad_split=None, need_dgrad=True, q_taps=9,
                 prev: BNState = None, first_x=None):
        """BN+ReLU backward then conv weight/bias grads and the data gradient. dg carries dA and the
        BN-backward sums its producer wrote. The data gradient comes back as a DGrad whose sums are
        those of `prev` (the CBR block that produced this layer's input), or a (d(up), d(skip))
        pair for a concatenated input (d(up) with its column sums)."""
        st: BNState = ctx.bn[name]
        M, co, dev = st.n * st.h * st.w, st.c, st.y.device
        coef = K.keep(torch.empty(3, co, dtype=torch.float32, device=dev))
        gamma = ctx.params[f"{name}.1.weight"]
        ws = K.keep(torch.empty(K.query("selunet_reduce_ws_bytes", 3 * co) // 8, dtype=torch.float64, device=dev))
        wp = ctx.wpack[name] if first_x is None else None
        ci = sum(s.channels for s in input_srcs)
        # the BN-backward apply fused into the split-fp16 weight gradient: dA's producer
        # recorded max |dA|, the finalize turns it into a bound of |dy|, the weight gradient forms dy from
        # (dA, y) while staging and writes it (with its exact max) for the data gradient
        # (a sums-only producer's dA, dg.src, at 64 channels: the pool / heads forms of the staging)
        src = dg.src if (dg.src is not None and co == 64 and self.fuse_wgrad_src) else None
        fuse = (wp is not None and wp.mode in X2_MODES and dg.da_word and self.fuse_wgrad_apply and
                (src is not None or (dg.apply is None and dg.t is not None)) and
                all(sr.amax is not None for sr in input_srcs))
        gp = gq = None
        if fuse:  # (with a src, p only gives the grid and channel count: y stands in for dA)
            gp = K.gather(st.n, st.h, st.w, 1, K.source(dg.t if src is None else st.y, co))
            gq = K.gather(st.n, st.h, st.w, q_taps, *input_srcs)
            fuse = K.query("selunet_conv3x3_wgrad_x2_ws_bytes", gp, gq) > 0
        if fuse:
            K.call("selunet_bn_bwd_stats_finalize_bound", K.ptr(dg.slab), dg.rows, K.ptr(ws), None, M, co, K.ptr(gamma),
                   K.ptr(st.invstd), K.ptr(G[f"{name}.1.weight"]), K.ptr(G[f"{name}.1.bias"]),
                   K.ptr(G[f"{name}.0.bias"]), K.ptr(coef), K.ptr(self._word(ctx, "da:" + name)),
                   K.ptr(self._word(ctx, "dyb:" + name)), self.stream)
        else:
            K.call("selunet_bn_bwd_stats_finalize", K.ptr(dg.slab), dg.rows, K.ptr(ws), None, M, co, K.ptr(gamma),
                   K.ptr(st.invstd), K.ptr(G[f"{name}.1.weight"]), K.ptr(G[f"{name}.1.bias"]),
                   K.ptr(G[f"{name}.0.bias"]), K.ptr(coef), self.stream)
        if first_x is not None:
            # encoder_layer_1_1: its dy feeds only the weight gradient (the input needs none), which
            # forms it from dA and y while staging (selunet_first_conv_wgrad_bn): dy is never written
            cin = first_x.shape[1]
            rows = K.query("selunet_first_conv_wgrad_rows", st.n, st.h, st.w)
            slab = K.keep(torch.empty(rows, co, FIRST_KPAD, dtype=torch.float32, device=dev))
            K.call("selunet_first_conv_wgrad_bn", K.ptr(first_x), st.n, cin, st.h, st.w, K.ptr(dg.t), K.ptr(st.y),
                   K.ptr(st.scale), K.ptr(st.shift), K.ptr(st.mean), K.ptr(st.invstd), K.ptr(coef), K.ptr(slab),
                   self.code, self.stream)
            packed = K.keep(torch.empty(co, FIRST_KPAD, dtype=torch.float32, device=dev))
            self._reduce(slab, rows, co * FIRST_KPAD, out32=packed)
            K.call("selunet_unpack_conv3x3_grad", K.ptr(packed), co, cin, FIRST_KPAD, K.ptr(G[f"{name}.0.weight"]),
                   self.stream)
            K.marker(("grads", name))
            return None
        dy = K.keep(torch.empty(M, co, dtype=self.dt, device=dev))
        dyw = self._word(ctx, "dy:" + name) if wp.mode in X2_MODES else None
        if fuse:
            # weight gradient with the apply in its dY staging; it writes dy and max |dy| (dyw)
            wsb = K.query("selunet_conv3x3_wgrad_x2_ws_bytes", gp, gq)
            wsx = K.keep(torch.empty(wsb // 4, dtype=torch.float32, device=dev))
            words = [sr.amax for sr in input_srcs]
            args = (gp, gq, K.ptr(wsx), wsb, K.ptr(G[f"{name}.0.weight"]), K.ptr(self._word(ctx, "dyb:" + name)),
                    K.ptr(words[0]), K.ptr(words[1]) if len(words) > 1 else None, bnb_for(st, None), K.ptr(coef))
            if src is not None:
                K.call("selunet_conv3x3_wgrad_x2_bn_src", *args, src, K.ptr(dy), K.ptr(dyw), self.stream)
            else:
                K.call("selunet_conv3x3_wgrad_x2_bn", *args, K.ptr(dy), K.ptr(dyw), self.stream)
        else:
            if dg.apply is not None:  # dA formed on the fly from its producer's inputs
                dg.apply(dy, coef, dyw)
            elif dyw is not None:  # dy with its range word (the split-fp16 data gradient reads it)
                K.call("selunet_bn_bwd_apply_amax", K.ptr(dg.t), K.ptr(st.y), M, co, K.ptr(st.scale),
                       K.ptr(st.shift), K.ptr(st.mean), K.ptr(st.invstd), K.ptr(coef), K.ptr(dy), K.ptr(dyw),
                       self.code, self.stream)
            else:
                K.call("selunet_bn_bwd_apply", K.ptr(dg.t), K.ptr(st.y), M, co, K.ptr(st.scale), K.ptr(st.shift),
                       K.ptr(st.mean), K.ptr(st.invstd), K.ptr(coef), K.ptr(dy), self.code, self.stream)
            # weight gradient: out[co][(tap, ci)] = sum_m dy[m][co] * X_im2col[m][(tap, ci)]
            ld = K.query("selunet_wgrad_ld", q_taps * ci)
            gp = K.gather(st.n, st.h, st.w, 1, K.source(dy, co))
            gq = K.gather(st.n, st.h, st.w, q_taps, *input_srcs)
            if not self._wgrad_x2(gp, gq, dyw, input_srcs, G[f"{name}.0.weight"]):
                self._wgrad_param(gp, gq, K.WG_CONV3X3, co, ld, G[f"{name}.0.weight"])
        K.marker(("grads", name))
        if not need_dgrad:
            return None
        wd = wp.dgrad
        dsrc = K.source(dy, co, amax=dyw)
        ga = K.gather(st.n, st.h, st.w, 9, dsrc)
        rows = (K.query("selunet_conv3x3_x2_stats_rows", ga, ci) if wp.mode in X2_MODES
                else K.query("selunet_gemm_stats_rows", ga, ci, self.code))
        if dgrad_split is None:
            dx = K.keep(torch.empty(M, ci, dtype=self.dt, device=dev))
            ep = K.Epilogue(K.ptr(dx), None, None, None, K.EP_PLAIN, 0)
            slab = None
            if prev is not None:
                slab = K.keep(torch.empty(rows, 3, ci, dtype=torch.float32, device=dev))
                ep.bnb = bnb_for(prev, slab)
                if ctx.x2 and ("da:" + prev.name) in ctx.words:  # max |dA| for a fused apply's |dy| bound
                    ep.amax = K.ptr(self._word(ctx, "da:" + prev.name))
            self._conv3x3(ga, wd, ci, 9 * co, ep, wp.mode, (dsrc,))
            return DGrad(dx, slab, rows, da_word=ep.amax is not None)
        c0 = dgrad_split
        d0 = K.keep(torch.empty(M, c0, dtype=self.dt, device=dev))
        d1 = K.keep(torch.empty(M, ci - c0, dtype=self.dt, device=dev))
        colsum = K.keep(torch.empty(rows, c0, dtype=torch.float32, device=dev))
        ep = K.Epilogue(K.ptr(d0), K.ptr(d1), None, None, K.EP_SPLIT, c0, K.ptr(colsum))
        if ctx.x2:  # a bound on d(up) (both halves' max): the split-fp16 ConvTranspose2d data gradient reads it
            ep.amax = K.ptr(self._word(ctx, "du:" + name))
        self._conv3x3(ga, wd, ci, 9 * co, ep, wp.mode, (dsrc,))
        return DGrad(d0, colsum, rows), d1

    def _up_bwd(self, ctx, name, du: DGrad, G, prev: BNState):
        """ConvTranspose2d(k2,s2) backward: bias (from du's column sums), weight and data gradients;
        the data gradient carries prev's BN-backward sums."""
        wp = ctx.wpack[name]
        wd, ci, co = wp.dgrad, wp.kpad, wp.co
        n, h, w = prev.n, prev.h, prev.w
        dev = du.t.device
        self._reduce(du.slab, du.rows, co, out32=G[f"{name}.bias"])
        ld = K.query("selunet_wgrad_ld", 4 * co)
        gp = K.gather(n, h, w, 1, prev.src())
        gq = K.gather(n, h, w, 4, K.source(du.t, co))
        duw = self._word(ctx, "du:decoder_layer_" + name[-1] + "_2") if wp.mode == "x2" else None
        wsb = K.query("selunet_gemm_wgrad_x2_ws_bytes", gp, gq) if duw is not None else -1
        if wsb > 0:  # split-fp16 weight gradient (unpool k feeds decoder_layer_k_2)
            ws = K.keep(torch.empty(wsb // 4, dtype=torch.float32, device=dev))
            K.call("selunet_gemm_wgrad_x2", gp, gq, K.ptr(ws), wsb, K.WG_CONVT, K.ptr(G[f"{name}.weight"]),
                   K.ptr(prev.amax), None, K.ptr(duw), None, self.stream)
        else:
            self._wgrad_param(gp, gq, K.WG_CONVT, ci, ld, G[f"{name}.weight"])
        K.marker(("grads", name))
        dz = K.keep(torch.empty(n * h * w, ci, dtype=self.dt, device=dev))
        ga = K.gather(n, h, w, 4, K.source(du.t, co))
        rows = (K.query("selunet_gemm_gather_x2_stats_rows", ga, ci) if wp.mode == "x2"
                else K.query("selunet_gemm_stats_rows", ga, ci, self.code))
        slab = K.keep(torch.empty(rows, 3, ci, dtype=torch.float32, device=dev))
        ep = K.Epilogue(K.ptr(dz), None, None, None, K.EP_PLAIN, 0)
        ep.bnb = bnb_for(prev, slab)
        da_word = False
        if wp.mode == "x2":
            if ("da:" + prev.name) in ctx.words:  # max |dA| for a fused apply's |dy| bound
                ep.amax = K.ptr(self._word(ctx, "da:" + prev.name))
                da_word = True
            K.call("selunet_gemm_gather_x2", ga, K.ptr(wd), ci, 4 * co, ep, K.ptr(duw), None, self.stream)
        else:
            K.call("selunet_gemm_gather", ga, K.ptr(wd), ci, 4 * co, ep, self.code, self.stream)
        return DGrad(dz, slab, rows, da_word=da_word)

    def _pool_bwd(self, ctx, st: BNState, dp: DGrad, dskip):
        rows = K.query("selunet_maxpool2_bwd_slab_rows", st.n, st.h, st.w, st.c)
        slab = K.keep(torch.empty(rows, 3, st.c, dtype=torch.float32, device=st.y.device))
        if K.fused_apply_enabled():  # the sums only; the layer's BN-backward apply routes dP itself
            word = ctx.words.get("da:" + st.name) if ctx.x2 else None  # max |dA| for the fused weight gradient
            K.call("selunet_maxpool2_bwd", K.ptr(st.y), st.n, st.h, st.w, st.c, K.ptr(st.scale), K.ptr(st.shift),
                   K.ptr(dp.t), K.ptr(dskip), None, bnb_for(st, slab, word), self.code, self.stream)

            def apply(dy, coef, word):
                K.call("selunet_bn_bwd_apply_pool", K.ptr(st.y), st.n, st.h, st.w, st.c, K.ptr(st.scale),
                       K.ptr(st.shift), K.ptr(st.mean), K.ptr(st.invstd), K.ptr(coef), K.ptr(dp.t), K.ptr(dskip),
                       K.ptr(dy), K.ptr(word), self.code, self.stream)
            src = K.DaSource(K.DA_POOL, 0, K.ptr(dp.t), K.ptr(dskip))
            return DGrad(None, slab, rows, apply, da_word=word is not None, src=src)
        bnb = bnb_for(st, slab)
        dz = K.keep(torch.empty_like(st.y))
        K.call("selunet_maxpool2_bwd", K.ptr(st.y), st.n, st.h, st.w, st.c, K.ptr(st.scale), K.ptr(st.shift),
               K.ptr(dp.t), K.ptr(dskip), K.ptr(dz), bnb, self.code, self.stream)
        return DGrad(dz, slab, rows)

    def backward(self, ctx, P, G, g_heads, flat, on_grads=None):
        """g_heads: list of fp32 [N,H,W] grads of (out[, select, aux]) (None -> zeros). G: the
        parameter-gradient views (reference layouts) of the flat fp32 buffer `flat`, written here.
        on_grads(layer_name) is called on the host as soon as a layer's parameter gradients are
        enqueued (heads first, encoder_layer_1_1 last), e.g. to start their all-reduce while the
        rest of the backward runs."""
        g_heads = [g.contiguous() if g is not None else None for g in g_heads]
        e = ctx.entry
        cb = (lambda tag: on_grads(tag[1])) if on_grads is not None else None
        if e is None:
            with K.marker_callback(cb):
                self._backward_impl(ctx, P, G, g_heads)
            return
        pattern = tuple(g is None for g in g_heads)
        slots = {"x": ctx.x, "flat": flat, **{f"g{i}": g for i, g in enumerate(g_heads) if g is not None}}
        plan = e.bwd.get(pattern)
        try:
            if plan is not None:
                plan.replay(slots, on_marker=cb)
            else:
                plan = K.Plan(slots)
                with K.recording(plan), K.marker_callback(cb):
                    self._backward_impl(ctx, P, G, g_heads)
                e.bwd[pattern] = plan
        finally:
            e.busy = False

    def _backward_impl(self, ctx, P, G, g_heads):
        ctx.params = P
        n, cin, H, W = ctx.shape
        M = n * H * W
        dev = ctx.x.device
        bn = ctx.bn
        heads = LY.HEADS if ctx.selective else LY.HEADS[:1]
        d11 = bn["decoder_layer_1_1"]
        rows = K.query("selunet_channel_slab_rows", M)
        bslab = K.keep(torch.empty(rows, 3, 64, dtype=torch.float32, device=dev))
        ce = getattr(ctx, "ce_heads", None)
        if ce is not None:
            heads = [h for h, _ in ce]
            gs = [g if g is not None else K.keep(torch.zeros(n, c, H, W, dtype=torch.float32, device=dev))
                  for g, (_, c) in zip(g_heads, ce)]
            planes = self._planes(gs, ce, H * W, with_slab=True)
            slab = K.keep(torch.empty(rows, planes.row_len, dtype=torch.float32, device=dev))
            fused = K.fused_apply_enabled()  # sums only: decoder_layer_1_1's apply forms dA from the planes
            dz = None if fused else K.keep(torch.empty(M, 64, dtype=self.dt, device=dev))
            K.call("selunet_heads_bwd_planes", K.ptr(d11.y), M, K.ptr(d11.scale), K.ptr(d11.shift), K.ptr(ctx.head_w),
                   planes, K.ptr(dz), K.ptr(slab), bnb_for(d11, bslab), self.code, self.stream)
            seg = planes.row_len
            head_w = ctx.head_w

            def apply_planes(dy, coef, word):
                K.call("selunet_bn_bwd_apply_heads_planes", K.ptr(d11.y), M, K.ptr(d11.scale), K.ptr(d11.shift),
                       K.ptr(d11.mean), K.ptr(d11.invstd), K.ptr(coef), K.ptr(head_w), planes, K.ptr(dy),
                       K.ptr(word), self.code, self.stream)
        else:
            gs = [g if g is not None else K.keep(torch.zeros(n, H, W, dtype=torch.float32, device=dev))
                  for g in g_heads]
            gs = gs + [None] * (3 - len(gs))
            nh = len(heads)
            slab = K.keep(torch.empty(rows, nh * 65, dtype=torch.float32, device=dev))
            fused = K.fused_apply_enabled()  # sums only: decoder_layer_1_1's apply forms dA from the g planes
            dz = None if fused else K.keep(torch.empty(M, 64, dtype=self.dt, device=dev))
            # max |dA| for the fused weight gradient (sums-only mode)
            hword = ctx.words.get("da:decoder_layer_1_1") if (ctx.x2 and fused) else None
            K.call("selunet_heads_bwd", K.ptr(d11.y), M, K.ptr(d11.scale), K.ptr(d11.shift), K.ptr(ctx.head_w), nh,
                   K.ptr(gs[0]), K.ptr(gs[1]), K.ptr(gs[2]), K.ptr(dz), K.ptr(slab), bnb_for(d11, bslab, hword),
                   self.code, self.stream)
            seg = nh * 65
        apply = apply_planes if (ce is not None and dz is None) else None
        hsrc = None
        if dz is None and ce is None:
            head_w = ctx.head_w

            def apply(dy, coef, word):
                K.call("selunet_bn_bwd_apply_heads", K.ptr(d11.y), M, K.ptr(d11.scale), K.ptr(d11.shift),
                       K.ptr(d11.mean), K.ptr(d11.invstd), K.ptr(coef), K.ptr(head_w), nh, K.ptr(gs[0]), K.ptr(gs[1]),
                       K.ptr(gs[2]), K.ptr(dy), K.ptr(word), self.code, self.stream)
            g3 = (ctypes.c_void_p * 3)(*[K.ptr(g) for g in gs[:3]])
            hsrc = K.DaSource(K.DA_HEADS, nh, None, None, K.ptr(head_w), g3)
        dz = DGrad(dz, bslab, rows, apply, da_word=hsrc is not None and hword is not None, src=hsrc)
        # the head weight/bias grads are one consecutive segment of the gradient buffer (registration
        # order conv1x1, conv_select, conv_aux; weight then bias each): reduce straight into it
        hw0 = G[f"{heads[0]}.weight"]
        off = 0
        for h in heads:
            assert G[f"{h}.weight"].data_ptr() == hw0.data_ptr() + off * 4
            off += G[f"{h}.weight"].numel()
            assert G[f"{h}.bias"].data_ptr() == hw0.data_ptr() + off * 4
            off += G[f"{h}.bias"].numel()
        assert off == seg
        self._reduce(slab, rows, seg, out32=hw0)
        K.marker(("grads", "heads"))

        e12, e22, e32 = bn["encoder_layer_1_2"], bn["encoder_layer_2_2"], bn["encoder_layer_3_2"]
        u1, u2, u3 = ctx.ups["unpool1"], ctx.ups["unpool2"], ctx.ups["unpool3"]
        p1, p2, p3 = ctx.pools["pool1"], ctx.pools["pool2"], ctx.pools["pool3"]
        cb = lambda name, d, srcs, **kw: self._cbr_bwd(ctx, name, d, G, srcs, **kw)  # noqa: E731
        uw = lambda nm: ctx.words.get("up:" + nm)  # noqa: E731  range words (split-fp16 layers)

        dz = cb("decoder_layer_1_1", dz, [bn["decoder_layer_1_2"].src()], prev=bn["decoder_layer_1_2"])
        du1, dskip1 = cb("decoder_layer_1_2", dz, [K.source(u1, 64, amax=uw("unpool1")), e12.src()],
                            dgrad_split=64)
        dz = self._up_bwd(ctx, "unpool1", du1, G, bn["decoder_layer_2_1"])
        dz = cb("decoder_layer_2_1", dz, [bn["decoder_layer_2_2"].src()], prev=bn["decoder_layer_2_2"])
        du2, dskip2 = cb("decoder_layer_2_2", dz, [K.source(u2, 128, amax=uw("unpool2")), e22.src()],
                            dgrad_split=128)
        dz = self._up_bwd(ctx, "unpool2", du2, G, bn["decoder_layer_3_1"])
        dz = cb("decoder_layer_3_1", dz, [bn["decoder_layer_3_2"].src()], prev=bn["decoder_layer_3_2"])
        du3, dskip3 = cb("decoder_layer_3_2", dz, [K.source(u3, 256, amax=uw("unpool3")), e32.src()],
                            dgrad_split=256)
        dz = self._up_bwd(ctx, "unpool3", du3, G, bn["decoder_layer_4_1"])
        dz = cb("decoder_layer_4_1", dz, [bn["decoder_layer_4_2"].src()], prev=bn["decoder_layer_4_2"])
        dp3 = cb("decoder_layer_4_2", dz, [K.source(p3, 256, amax=e32.amax)])
        dz = self._pool_bwd(ctx, e32, dp3, dskip3)
        dz = cb("encoder_layer_3_2", dz, [bn["encoder_layer_3_1"].src()], prev=bn["encoder_layer_3_1"])
        dp2 = cb("encoder_layer_3_1", dz, [K.source(p2, 128, amax=e22.amax)])
        dz = self._pool_bwd(ctx, e22, dp2, dskip2)
        dz = cb("encoder_layer_2_2", dz, [bn["encoder_layer_2_1"].src()], prev=bn["encoder_layer_2_1"])
        dp1 = cb("encoder_layer_2_1", dz, [K.source(p1, 64, amax=e12.amax)])
        dz = self._pool_bwd(ctx, e12, dp1, dskip1)
        dz = cb("encoder_layer_1_2", dz, [bn["encoder_layer_1_1"].src()], prev=bn["encoder_layer_1_1"])
        cb("encoder_layer_1_1", dz, [], need_dgrad=False, first_x=ctx.x)
