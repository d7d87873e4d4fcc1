"""Helpers to read the golden fixtures written by tests/golden/make_golden.py and
compare a candidate (oracle or HIP path) against them."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


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


def check_grads_vs_truth(d, grads, floor=1e-2, factor=3.0, skip=()):
    """Gradient parity measured against the reference's own fp64 run (`s0/grad64*`).

    ReLU masks and max-pool argmaxes make the gradient a discontinuous function of the
    forward values: an element within rounding of a kink routes its gradient differently in
    any two fp32 implementations (the reference's own fp32 gradients deviate from its fp64 run
    by up to 5.6% of a tensor's max on these fixtures, and by ~1e-6 where no element happens to
    flip). So the bound is statistical: per tensor, the relative L2 error over the fixture's
    samples, e = ||g - g64|| / ||g64||, must satisfy e_ours <= max(floor, factor * e_ref32);
    same for the full-tensor norm. A layout or indexing bug gives e = O(1).
    Returns (failures, report) with report = (name, e_ours, e_ref) sorted by e_ours."""
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
        report.append((name, e_ours, e_ref))
        if e_ours > max(floor, factor * e_ref):
            fails.append(f"{name}: sample err vs fp64 {e_ours:.2e} > max({floor:g}, {factor:g} x ref {e_ref:.2e})")
        if en_ours > max(floor, factor * en_ref):
            fails.append(f"{name}: norm err vs fp64 {en_ours:.2e} > max({floor:g}, {factor:g} x ref {en_ref:.2e})")
    report.sort(key=lambda r: -r[1])
    return fails, report
