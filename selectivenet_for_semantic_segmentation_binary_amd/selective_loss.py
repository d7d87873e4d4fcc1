"""Selective risk and aux BCE on the MI355X (reference: selective_loss.py:58-85, train.py:78,195).

`calc_selective_risk_image_b(output, selection, target, target_coverage=0.8, lamb=8,
hard_selection=False) -> (loss, coverage)` keeps the reference signature and return values:

    s = sigmoid(selection); coverage = mean(s)
    risk = -mean((t*log(sigmoid(x)) + (1-t)*log(1-sigmoid(x))) * s) / coverage
    loss = risk + lamb * max(target_coverage - coverage, 0)^2

computed by wavefront-reduced HIP kernels (partials -> deterministic fp64 reduce -> scalar
finalize) with log(sigmoid(x)) = -softplus(-x) and log(1-sigmoid(x)) = -softplus(x). This equals
the reference wherever the reference is finite; the reference's literal fp32 form returns NaN as
soon as a logit saturates (|x| > ~16.6) and loses digits from |x| ~ 9 on.

Under data parallelism (parallel.init_data_parallel) the partial sums are all-reduced, so loss
and coverage are those of the global batch — what DataParallel computes after gathering the
outputs to cuda:0 — and each rank back-propagates its own pixels with the global normalisers.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as K
from . import parallel


def _check(t, name):
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a cuda tensor (the MI355X losses have no CPU fallback)")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _reduced_sums(slab, rows, cols):
    """fp64 column sums of a partial slab, all-reduced across data-parallel ranks."""
    sums = torch.empty(cols, dtype=torch.float64, device=slab.device)
    ws = torch.empty(K.query("selunet_reduce_ws_bytes", cols) // 8, dtype=torch.float64, device=slab.device)
    K.call("selunet_reduce_rows", K.ptr(slab), rows, cols, K.ptr(ws), K.ptr(sums), None, K.stream_ptr())
    parallel.allreduce_sums(sums)
    return sums


def _global_count(p_local: int) -> float:
    t = torch.tensor([float(p_local)], dtype=torch.float64,
                     device="cuda" if torch.cuda.is_available() else "cpu")
    parallel.allreduce_sums(t)
    return float(t.item())


def global_count(shape) -> float:
    """Global pixel count of the data-parallel batch whose local part has `shape` (N, H, W).

    With the global batch registered (parallel.set_global_batch / parallel.local_batch) it is
    B * H * W with no exchange; otherwise one all-reduce of the local count, every call — never
    cached, since ranks may hold chunks of different sizes (torch.chunk of a ragged last batch)
    and a rank answering from a cache while another all-reduces would deadlock."""
    p_local = 1
    for d in shape:
        p_local *= int(d)
    if not parallel.is_initialized():
        return float(p_local)
    b = parallel.global_batch()
    if b is not None and int(shape[0]) > 0:
        return float(b * (p_local // int(shape[0])))
    return _global_count(p_local)


class _SelectiveRiskB(torch.autograd.Function):
    @staticmethod
    def forward(ctx, output, selection, target, target_coverage, lamb, hard=False):
        p = output.numel()
        dev = output.device
        rows = K.query("selunet_loss_slab_rows", p)
        slab = torch.empty(rows, 2, dtype=torch.float32, device=dev)
        K.call("selunet_selective_partials_hard" if hard else "selunet_selective_partials", K.ptr(output),
               K.ptr(selection), K.ptr(target), p, K.ptr(slab), K.stream_ptr())
        sums = _reduced_sums(slab, rows, 2)
        p_global = global_count(output.shape)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        coverage = torch.empty((), dtype=torch.float32, device=dev)
        state = torch.empty(4, dtype=torch.float32, device=dev)
        K.call("selunet_selective_finalize", K.ptr(sums), p_global, float(lamb), float(target_coverage), K.ptr(loss),
               K.ptr(coverage), K.ptr(state), K.stream_ptr())
        ctx.save_for_backward(output, selection, target, state)
        ctx.lamb, ctx.hard = float(lamb), hard
        if hard:
            ctx.mark_non_differentiable(coverage)  # coverage.clone().detach(), selective_loss.py:76
        return loss, coverage

    @staticmethod
    def backward(ctx, g_loss, g_cov):
        output, selection, target, state = ctx.saved_tensors
        d_out = torch.empty_like(output)
        d_sel = torch.empty_like(selection)
        gl = g_loss.contiguous().float() if g_loss is not None else None
        gc = g_cov.contiguous().float() if g_cov is not None else None
        if ctx.hard:  # selection detached: no gradient reaches it (d_sel is written as zeros)
            K.call("selunet_selective_bwd_hard", K.ptr(output), K.ptr(selection), K.ptr(target), output.numel(),
                   K.ptr(state), K.ptr(gl), K.ptr(d_out), K.ptr(d_sel), K.stream_ptr())
            return d_out, None, None, None, None, None
        K.call("selunet_selective_bwd", K.ptr(output), K.ptr(selection), K.ptr(target), output.numel(), K.ptr(state),
               ctx.lamb, K.ptr(gl), K.ptr(gc), K.ptr(d_out), K.ptr(d_sel), K.stream_ptr())
        return d_out, d_sel, None, None, None, None


def calc_selective_risk_image_b(output, selection, target, target_coverage=0.8, lamb=8, hard_selection=False):
    """selective_loss.py:58-85 (BCE-with-logits selective risk). output/selection/target: (N, H, W).

    hard_selection=True (selective_loss.py:74-77): the risk's selection weight is the detached
    [sigmoid(g) > 0.5], the coverage the detached soft mean — the loss then reaches `output` only."""
    if output.shape != selection.shape or output.shape != target.shape:
        raise ValueError(f"shape mismatch: output {tuple(output.shape)}, selection {tuple(selection.shape)}, "
                         f"target {tuple(target.shape)}")
    o, s, t = _check(output, "output"), _check(selection, "selection"), _check(target, "target")
    return _SelectiveRiskB.apply(o, s, t, target_coverage, lamb, bool(hard_selection))


class _BCEWithLogitsMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logit, target):
        p = logit.numel()
        dev = logit.device
        rows = K.query("selunet_loss_slab_rows", p)
        slab = torch.empty(rows, 1, dtype=torch.float32, device=dev)
        K.call("selunet_bce_partials", K.ptr(logit), K.ptr(target), p, K.ptr(slab), K.stream_ptr())
        sums = _reduced_sums(slab, rows, 1)
        p_global = global_count(logit.shape)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        K.call("selunet_bce_finalize", K.ptr(sums), p_global, K.ptr(loss), K.stream_ptr())
        ctx.save_for_backward(logit, target)
        ctx.p_global = p_global
        return loss

    @staticmethod
    def backward(ctx, g):
        logit, target = ctx.saved_tensors
        d = torch.empty_like(logit)
        g = g.contiguous().float()  # keep alive until the launch is enqueued
        K.call("selunet_bce_bwd", K.ptr(logit), K.ptr(target), logit.numel(), ctx.p_global, K.ptr(g), K.ptr(d),
               K.stream_ptr())
        return d, None


class BCEWithLogitsLoss(nn.Module):
    """torch.nn.BCEWithLogitsLoss() with the default reduction='mean' (train.py:78)."""

    def __init__(self, weight=None, size_average=None, reduce=None, reduction="mean", pos_weight=None):
        super().__init__()
        if weight is not None or pos_weight is not None or reduction != "mean" or size_average is not None \
                or reduce is not None:
            raise NotImplementedError("only the reference's BCEWithLogitsLoss() (mean, unweighted) is implemented")

    def forward(self, input, target):
        if input.shape != target.shape:
            raise ValueError(f"Target size ({tuple(target.shape)}) must be the same as input size "
                             f"({tuple(input.shape)})")
        return _BCEWithLogitsMean.apply(_check(input, "input"), _check(target, "target"))


# ----------------------------------------------------------------------------- CE forms (CE UNet)
def _check_target_ce(target, logits):
    if target.device.type != "cuda":
        raise RuntimeError("target must be a cuda tensor (the MI355X losses have no CPU fallback)")
    if target.dtype != torch.int64:
        raise RuntimeError(f"expected int64 class indices as target (got {target.dtype})")
    n, c, h, w = logits.shape
    if tuple(target.shape) != (n, h, w):
        raise ValueError(f"target {tuple(target.shape)} must be (N, H, W) = {(n, h, w)} for logits "
                         f"{tuple(logits.shape)}")
    if c > 8:
        raise ValueError(f"at most 8 classes on the MI355X path (got {c})")
    return target.contiguous()


class _SelectiveRiskCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, output, selection, target, target_coverage, lamb, hard=False):
        n, c, h, w = output.shape
        hw, p = h * w, n * h * w
        dev = output.device
        rows = K.query("selunet_loss_slab_rows", p)
        slab = torch.empty(rows, 2, dtype=torch.float32, device=dev)
        K.call("selunet_ce_selective_partials_hard" if hard else "selunet_ce_selective_partials", K.ptr(output), K.ptr(selection), K.ptr(target), n, c, hw, K.ptr(slab),
               K.stream_ptr())
        sums = _reduced_sums(slab, rows, 2)
        p_global = global_count((n, h, w))
        loss = torch.empty((), dtype=torch.float32, device=dev)
        coverage = torch.empty((), dtype=torch.float32, device=dev)
        state = torch.empty(4, dtype=torch.float32, device=dev)
        K.call("selunet_selective_finalize", K.ptr(sums), p_global, float(lamb), float(target_coverage), K.ptr(loss),
               K.ptr(coverage), K.ptr(state), K.stream_ptr())
        ctx.save_for_backward(output, selection, target, state)
        ctx.lamb, ctx.hard = float(lamb), hard
        if hard:
            ctx.mark_non_differentiable(coverage)  # selective_loss.py:47
        return loss, coverage

    @staticmethod
    def backward(ctx, g_loss, g_cov):
        output, selection, target, state = ctx.saved_tensors
        n, c, h, w = output.shape
        d_out = torch.empty_like(output)
        d_sel = torch.empty_like(selection)
        gl = g_loss.contiguous().float() if g_loss is not None else None
        gc = g_cov.contiguous().float() if g_cov is not None else None
        if ctx.hard:
            K.call("selunet_ce_selective_bwd_hard", K.ptr(output), K.ptr(selection), K.ptr(target), n, c, h * w,
                   K.ptr(state), K.ptr(gl), K.ptr(d_out), K.ptr(d_sel), K.stream_ptr())
            return d_out, None, None, None, None, None
        K.call("selunet_ce_selective_bwd", K.ptr(output), K.ptr(selection), K.ptr(target), n, c, h * w, K.ptr(state),
               ctx.lamb, K.ptr(gl), K.ptr(gc), K.ptr(d_out), K.ptr(d_sel), K.stream_ptr())
        return d_out, d_sel, None, None, None, None


def calc_selective_risk_image(output, selection, target, target_coverage=0.8, lamb=8, hard_selection=False):
    """selective_loss.py:24-56 (cross-entropy selective risk, CE `UNet`): output (N, C, H, W),
    selection (N, 2, H, W), target (N, H, W) int64 class indices.

        s = softmax(selection, 1)[:, 1]; coverage = mean(s)
        risk = -mean(sum_c log_softmax(output, 1) * onehot(target) * s) / coverage
        loss = risk + lamb * max(target_coverage - coverage, 0)^2

    (the reference's one-hot target (N, C, H, W) form is accepted too and reduced to indices).
    hard_selection=True (selective_loss.py:43-48): detached [s > 0.5] weights, detached coverage."""
    if output.dim() != 4 or selection.dim() != 4 or selection.shape[1] != 2 or \
            selection.shape[0] != output.shape[0] or selection.shape[2:] != output.shape[2:]:
        raise ValueError(f"expected output (N, C, H, W) and selection (N, 2, H, W); got {tuple(output.shape)}, "
                         f"{tuple(selection.shape)}")
    if target.dim() == 4:  # one-hot (N, C, H, W) as selective_loss.py:36-37 builds it
        target = target.argmax(1)
    o, s = _check(output, "output"), _check(selection, "selection")
    return _SelectiveRiskCE.apply(o, s, _check_target_ce(target, o), target_coverage, lamb, bool(hard_selection))


class _CrossEntropyMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logit, target):
        n, c, h, w = logit.shape
        p = n * h * w
        dev = logit.device
        rows = K.query("selunet_loss_slab_rows", p)
        slab = torch.empty(rows, 1, dtype=torch.float32, device=dev)
        K.call("selunet_ce_partials", K.ptr(logit), K.ptr(target), n, c, h * w, K.ptr(slab), K.stream_ptr())
        sums = _reduced_sums(slab, rows, 1)
        p_global = global_count((n, h, w))
        loss = torch.empty((), dtype=torch.float32, device=dev)
        K.call("selunet_bce_finalize", K.ptr(sums), p_global, K.ptr(loss), K.stream_ptr())
        ctx.save_for_backward(logit, target)
        ctx.p_global = p_global
        return loss

    @staticmethod
    def backward(ctx, g):
        logit, target = ctx.saved_tensors
        n, c, h, w = logit.shape
        d = torch.empty_like(logit)
        g = g.contiguous().float()
        K.call("selunet_ce_bwd", K.ptr(logit), K.ptr(target), n, c, h * w, ctx.p_global, K.ptr(g), K.ptr(d),
               K.stream_ptr())
        return d, None


class CrossEntropyLoss(nn.Module):
    """torch.nn.CrossEntropyLoss() with the defaults the reference uses (train.py:80): mean over
    pixels, (N, C, H, W) logits, (N, H, W) int64 targets, no weights / smoothing. A target outside
    [0, C) (torch's ignore_index pixels included) makes the loss and its gradient NaN rather than
    being clamped into a class."""

    def __init__(self, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean",
                 label_smoothing=0.0):
        super().__init__()
        if weight is not None or size_average is not None or reduce is not None or reduction != "mean" \
                or label_smoothing != 0.0:
            raise NotImplementedError("only the reference's CrossEntropyLoss() (mean, unweighted) is implemented")
        if ignore_index != -100:
            raise NotImplementedError("ignore_index: the reference's labels are class indices 0..C-1 only "
                                      "(utils/data_utils.py:220-221); targets outside [0, C) give a NaN loss")
        self.ignore_index = ignore_index

    def forward(self, input, target):
        if input.dim() != 4:
            raise ValueError(f"expected (N, C, H, W) logits, got {tuple(input.shape)}")
        t = _check_target_ce(target, input)
        return _CrossEntropyMean.apply(_check(input, "input"), t)
