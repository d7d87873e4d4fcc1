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
