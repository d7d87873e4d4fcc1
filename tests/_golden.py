"""Helpers to read the golden fixtures written by tests/golden/make_golden.py and
compare a candidate (oracle or HIP path) against them."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# one line per fixture run (fixture, fp32 conv path, loss error, worst gradient error, mask flips),
# printed by tests/conftest.py::pytest_terminal_summary so a quiet run's tail carries them
SUMMARY = []


def format_summary(info):
    wg = info.get("worst_grad")
    g = f"worst grad rel-L2 {wg[1]:.2e} ({wg[0]}, {wg[2]})" if wg else "worst grad n/a"
    flips = info.get("mask_flips")
    near0 = info.get("near0")
    m = "mask flips n/a" if flips is None else (
        f"mask flips {flips}" + (f" (ref logits within 1e-6: {near0})" if near0 is not None else ""))
    return (f"{info.get('fixture', '?')} [{info.get('path', '?')}]: loss rel err {info.get('loss_rel_err', float('nan')):.2e}, "
            f"{g}, {m}")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def tensor_keys(d, prefix):
    """Names of tensors recorded under `<prefix>norm/<name>`."""
    p = prefix + "norm/"
    return [k[len(p):] for k in d.files if k.startswith(p)]


def check_tensors(d, prefix, named, rtol, atol, skip=(), atol_by_name=None):
    """Compare dict name->np.ndarray against fixture samples. Returns list of failures."""
    fails = []
    for name in tensor_keys(d, prefix):
        if name in skip:
            continue
        a = np.asarray(named[name], dtype=np.float64).ravel()
        at = (atol_by_name or {}).get(name, atol)
        if prefix + "full/" + name in d.files:
            ref = d[prefix + "full/" + name].astype(np.float64)
            got = a
        else:
            idx = d[prefix + "idx/" + name]
            ref = d[prefix + "val/" + name].astype(np.float64)
            got = a[idx]
        nref = float(d[prefix + "norm/" + name])
        ngot = float(np.linalg.norm(a))
        scale = max(np.abs(ref).max(), 1e-30)
        err = np.abs(got - ref)
        if not np.all(err <= at + rtol * scale):
            fails.append(f"{prefix}{name}: max err {err.max():.3e} (scale {scale:.3e})")
        if abs(ngot - nref) > at * np.sqrt(a.size) + rtol * nref:
            fails.append(f"{prefix}{name}: norm {ngot:.6e} vs {nref:.6e}")
    return fails


def max_rel(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


def grad_bound(e_ref, e_ens=0.0):
    """Allowed relative-L2 gradient error against the fp64 truth.

    e_ref: the reference fp32 run's error on the same samples; e_ens: the largest error of the
    reference's fp32 runs under rounding-level perturbations — of the input (`s0/grad_ens/<name>`,
    tests/golden/make_golden.py::augment_ensemble) and, where the fixture has it, of every
    convolution output (3e-7 relative, the measured rounding of the fp32 Winograd F(2,3)
    convolution: `s0/grad_ens_conv/<name>`, augment_conv_noise), whichever is larger. ReLU-mask / max-pool-argmax flips make the fp32
    gradient a discontinuous function of rounding noise, so one reference run's error is one draw:
    the same 1e-7 input perturbation moves the reference's own error on a tensor from 1e-6 to 1e-3
    (DESIGN.md §4). Bound: max(1e-4, 10 e_ref, 3 e_ens) — for a tensor no perturbation disturbs
    (e_ens < 1e-5) that is max(1e-4, 10 e_ref)."""
    return max(1e-4, 10.0 * e_ref, 3.0 * e_ens)


def check_grads_vs_truth(d, grads, skip=(), bound=grad_bound):
    """Gradient parity measured against the reference's own fp64 run (`s0/grad64*`).

    ReLU masks and max-pool argmaxes make the gradient a discontinuous function of the
    forward values: an element within rounding of a kink routes its gradient differently in
    any two fp32 implementations (the reference's own fp32 gradients deviate from its fp64 run
    by up to 5.6% of a tensor's max on these fixtures, and by ~1e-6 where no element happens to
    flip). So the bound is statistical: per tensor, the relative L2 error over the fixture's
    samples, e = ||g - g64|| / ||g64||, must satisfy e_ours <= grad_bound(e_ref32, e_ens); same
    for the full-tensor norm. A layout or indexing bug gives e = O(1).
    Returns (failures, report) with report = (name, e_ours, e_ref, e_ens) sorted by e_ours."""
    fails, report = [], []
    for name in tensor_keys(d, "s0/grad"):
        if name in skip:
            continue
        a = np.asarray(grads[name], np.float64).ravel()
        if "s0/gradfull/" + name in d.files:
            ref32 = d["s0/gradfull/" + name].astype(np.float64)
            g64 = d["s0/grad64full/" + name]
            got = a
        else:
            idx = d["s0/gradidx/" + name]
            ref32 = d["s0/gradval/" + name].astype(np.float64)
            g64 = d["s0/grad64val/" + name]
            got = a[idx]
        scale = max(np.linalg.norm(g64), 1e-30)
        e_ref = float(np.linalg.norm(ref32 - g64) / scale)
        e_ours = float(np.linalg.norm(got - g64) / scale)
        n64 = float(d["s0/grad64norm/" + name])
        n_ref = float(d["s0/gradnorm/" + name])
        en_ref = abs(n_ref - n64) / max(n64, 1e-30)
        en_ours = abs(float(np.linalg.norm(a)) - n64) / max(n64, 1e-30)
        e_ens = max([float(d[k]) for k in ("s0/grad_ens/" + name, "s0/grad_ens_conv/" + name) if k in d.files],
                    default=0.0)
        report.append((name, e_ours, e_ref, e_ens))
        if e_ours > bound(e_ref, e_ens):
            fails.append(f"{name}: sample err vs fp64 {e_ours:.2e} > {bound(e_ref, e_ens):.2e} "
                         f"(reference fp32 {e_ref:.2e}, perturbed {e_ens:.2e})")
        if en_ours > bound(en_ref, e_ens):
            fails.append(f"{name}: norm err vs fp64 {en_ours:.2e} > {bound(en_ref, e_ens):.2e} "
                         f"(reference fp32 {en_ref:.2e}, perturbed {e_ens:.2e})")
    report.sort(key=lambda r: -r[1])
    return fails, report


def check_grads_vs_ref32(d, grads, bound, skip=()):
    """Gradients against the reference's fp32 run only (fixtures too large for an fp64 run):
    relative L2 error over the samples and of the full-tensor norm, each <= max(bound, 3 s) where
    s is the spread of the reference's own fp32 runs under rounding-level input perturbations
    (`s0/grad_spread/<name>`, augment_ensemble).
    Returns (failures, report) with report = (name, e_samples, e_norm, spread) sorted by e_samples."""
    fails, report = [], []
    for name in tensor_keys(d, "s0/grad"):
        if name in skip:
            continue
        a = np.asarray(grads[name], np.float64).ravel()
        if "s0/gradfull/" + name in d.files:
            ref, got = d["s0/gradfull/" + name].astype(np.float64), a
        else:
            ref, got = d["s0/gradval/" + name].astype(np.float64), a[d["s0/gradidx/" + name]]
        e = float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
        nref = float(d["s0/gradnorm/" + name])
        en = abs(float(np.linalg.norm(a)) - nref) / max(nref, 1e-30)
        sp = float(d["s0/grad_spread/" + name]) if "s0/grad_spread/" + name in d.files else 0.0
        b = max(bound, 3.0 * sp)
        report.append((name, e, en, sp))
        if e > b or en > b:
            fails.append(f"{name}: err vs reference fp32 {e:.2e} (norm {en:.2e}) > {b:.2e} (spread {sp:.2e})")
    report.sort(key=lambda r: -r[1])
    return fails, report


def mask_flips(d, pre, head, logits, tol):
    """Training-rule prediction-mask parity (train.py:150,153: fp64 sigmoid > 0.5) of one head.

    Returns (flips, near0): the number of pixels whose mask bit differs from the reference's, and
    the number of reference logits within 1e-6 of the decision boundary. Needs the fixture's full
    logits or its packed mask bits (`<head>_mask_bits`, with the sampled logits `<head>_idx/_val`).
    A flip is accepted only where the reference logit lies within the logit error this run measures
    on the same fixture: with full logits, |ref| at every flipped pixel <= the largest |ours - ref| over
    the pixels that did not flip; with packed bits, |ours| at every flipped pixel (>= |ref| - error
    there, and for a flip |ours| <= |ours - ref|) <= twice the largest |ours - ref| over the fixture's
    logit samples (16384 of 8.4M pixels at batch 128, so their maximum sits in the error tail but
    not necessarily at its end). `tol` (relative to the reference's max |logit|) caps both."""
    from oracle import unet_b_cpu as O  # (test infrastructure: the checker's threshold rule)

    logits = np.asarray(logits, np.float32)
    ours = O.train_pred_mask(logits).ravel()
    if pre + head in d.files:
        ref_logits = d[pre + head].astype(np.float32)
        ref = O.train_pred_mask(ref_logits).ravel()
        near0 = int((np.abs(ref_logits) < 1e-6).sum())
        absmax = float(np.abs(ref_logits).max())
        diff = ours != ref
        err = np.abs(logits.ravel().astype(np.float64) - ref_logits.ravel())
        e_meas = float(err[~diff].max(initial=0.0))
        at, bound = np.abs(ref_logits.ravel()), e_meas
    else:
        ref = np.unpackbits(d[pre + head + "_mask_bits"])[:ours.size]
        near0 = int(d[pre + head + "_near0_count"])
        absmax = float(d[pre + head + "_absmax"])
        diff = ours != ref
        idx = d[pre + head + "_idx"]
        e_meas = float(np.abs(logits.ravel()[idx].astype(np.float64) - d[pre + head + "_val"]).max())
        at, bound = np.abs(logits.ravel()), 2.0 * e_meas
    flips = int(diff.sum())
    if flips:
        worst = float(at[diff].max())
        assert worst <= min(bound, tol * absmax), (head, flips, worst, "measured logit error", e_meas, absmax)
    return flips, near0


def grad_errors(d, grads, skip=()):
    """Per tensor, the relative L2 error of `grads` on the fixture's samples against its truth: the
    fp64 step where the fixture has one, the reference's fp32 step otherwise (batch 128)."""
    has64 = any(k.startswith("s0/grad64norm/") for k in d.files)
    out = {}
    for name in tensor_keys(d, "s0/grad"):
        if name in skip:
            continue
        a = np.asarray(grads[name], np.float64).ravel()
        full = "s0/gradfull/" + name in d.files
        if has64:
            ref = d[("s0/grad64full/" if full else "s0/grad64val/") + name].astype(np.float64)
        else:
            ref = d[("s0/gradfull/" if full else "s0/gradval/") + name].astype(np.float64)
        got = a if full else a[d["s0/gradidx/" + name]]
        out[name] = float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
    return out
