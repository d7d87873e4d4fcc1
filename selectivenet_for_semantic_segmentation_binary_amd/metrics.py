"""On-device training/eval metrics: the per-batch host code of
train.py:211-238 and eval.py:218-246 plus `Evaluator` (utils/compute_metric.py:4-80), with the
[N,H,W] outputs never leaving HBM.

The reference copies every batch's logits to the host, applies a sigmoid in numpy and
thresholds it: `fn_classifier(fn_sigmoid(x))` = `1/(1+exp(-x)) > 0.5`, in float64 during
training (train.py:150,220-221) and in float32 with `--cut_off` / `--s_cut_off` at eval
(eval.py:171,175,230-231,238-240). Both rules are monotone in the fp32 logit, so each equals
`logit >= t` for one fp32 threshold `t`; `logit_threshold` finds that `t` once on the host by
bisection over the ordered fp32 values, evaluating the reference's own numpy expression (so
masks are bit-exact by construction; e.g. t = 1.5612511e-16 for the training rule and
1.2318974e-07 for the eval rule at cut_off 0.5). The device then only
compares and counts (`selunet_seg_metrics`): the 2x2 confusion matrix over selected pixels and
the selected/total pixel counts, accumulated as uint64 across batches.
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from . import _lib as K
from . import parallel


def _ordered(i: int) -> np.float32:
    """fp32 value with rank i in the total order of finite floats (i in [-2^31+2^23.., ...])."""
    if i >= 0:
        return np.array([i], np.int32).view(np.float32)[0]
    return -np.array([-i], np.int32).view(np.float32)[0]


def _rank(f: np.float32) -> int:
    b = int(np.array([f], np.float32).view(np.int32)[0])
    return b if b >= 0 else -(b & 0x7FFFFFFF)


@functools.lru_cache(maxsize=None)
def logit_threshold(rule: str = "train", cut_off: float = 0.5, output_scale: str = "sigmoid") -> float:
    """Smallest fp32 logit x with reference-pred(x) == 1.

    rule 'train': train.py:150,217-221 — fn_sigmoid in float64, then `> 0.5` (fn_classifier,
                  train.py:154); cut_off is fixed at 0.5 there.
    rule 'eval':  eval.py:171,175,229-231 — fn_sigmoid on the float32 array, `> cut_off`.
    output_scale != 'sigmoid': the raw logit is compared (`> cut_off`).
    """
    if rule == "argmax":
        # CE UNet with 2 classes (train.py:207-209, 216-219: np.argmax over the class / selection
        # axis, ties -> class 0): callers pass the fp32 difference x1 - x0, which is > 0 exactly
        # when x1 > x0; the smallest positive fp32 makes `>= t` the strict comparison.
        return float(np.nextafter(np.float32(0), np.float32(1)))
    if output_scale != "sigmoid":
        pred = lambda x: bool(np.array([x], np.float32) > cut_off)  # noqa: E731
    elif rule == "train":
        pred = lambda x: bool((1 / (1 + np.exp(-np.array([x], np.float32).astype("float64")))) > 0.5)  # noqa: E731
    elif rule == "eval":
        pred = lambda x: bool((1 / (1 + np.exp(-np.array([x], np.float32)))) > cut_off)  # noqa: E731
    else:
        raise ValueError(f"unknown threshold rule {rule!r}")
    with np.errstate(over="ignore"):
        return _bisect(pred)


def _bisect(pred) -> float:
    lo, hi = _rank(np.float32(-np.finfo(np.float32).max)), _rank(np.float32(np.finfo(np.float32).max))
    if pred(_ordered(lo)):
        return float(-np.inf)
    if not pred(_ordered(hi)):
        return float(np.inf)
    while hi - lo > 1:  # invariant: pred(lo) false, pred(hi) true
        mid = (lo + hi) // 2
        if pred(_ordered(mid)):
            hi = mid
        else:
            lo = mid
    return float(_ordered(hi))


class SegMetrics:
    """Device-side Evaluator (utils/compute_metric.py:4-80) for num_class = 2.

    add_batch(output, target, selection=None) counts one batch without a host copy;
    confusion_matrix() syncs once (and all-reduces across data-parallel ranks).
    """

    def __init__(self, device, selective: bool, rule: str = "train", cut_off: float = 0.5,
                 s_cut_off: float = 0.5, output_scale: str = "sigmoid"):
        self.selective = selective
        self.t_out = logit_threshold(rule, cut_off, output_scale)
        self.t_sel = logit_threshold(rule, s_cut_off, output_scale)
        self.counts = torch.zeros(6, dtype=torch.int64, device=device)  # uint64 bits

    def reset(self):
        self.counts.zero_()

    def add_batch(self, output: torch.Tensor, target: torch.Tensor, selection: torch.Tensor | None = None):
        for name, t in (("output", output), ("target", target), ("selection", selection)):
            if t is not None and (t.device.type != "cuda" or t.dtype != torch.float32 or not t.is_contiguous()):
                raise RuntimeError(f"SegMetrics.add_batch: {name} must be a contiguous cuda fp32 tensor")
        if output.numel() != target.numel() or (selection is not None and selection.numel() != output.numel()):
            raise ValueError("SegMetrics.add_batch: output, target and selection must have the same size")
        if self.selective and selection is None:
            raise ValueError("selective Evaluator needs the selection logits")
        sel = selection if self.selective else None
        K.call("selunet_seg_metrics", K.ptr(output), K.ptr(sel), K.ptr(target), output.numel(), self.t_out,
               self.t_sel, K.ptr(self.counts), K.stream_ptr())

    def raw(self) -> np.ndarray:
        c = self.counts.clone()
        parallel.allreduce_sums(c)
        return c.cpu().numpy().astype(np.int64)

    def confusion_matrix(self) -> np.ndarray:
        return self.raw()[:4].reshape(2, 2).astype(np.float64)

    def selected_total(self) -> tuple[int, int]:
        r = self.raw()
        return int(r[4]), int(r[5])


# Evaluator formulas (utils/compute_metric.py:34-80) on a host confusion matrix
def pixel_accuracy(cm):
    return np.diag(cm).sum() / cm.sum()


def mean_iou(cm):
    with np.errstate(invalid="ignore", divide="ignore"):
        iou = np.diag(cm) / (np.sum(cm, axis=1) + np.sum(cm, axis=0) - np.diag(cm))
    return np.nanmean(iou)


def precision(cm):
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.diag(cm) / cm.sum(axis=0)


def recall(cm):
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.diag(cm) / cm.sum(axis=1)


def dice(cm):
    with np.errstate(invalid="ignore", divide="ignore"):
        return 2 * np.diag(cm) / (np.sum(cm, axis=1) + np.sum(cm, axis=0))
