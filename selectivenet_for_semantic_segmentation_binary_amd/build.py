"""Build libselunet.so (all HIP kernels + the C-ABI) in-tree for gfx950 with hipcc.

    python -m selectivenet_for_semantic_segmentation_binary_amd.build [--force]

Objects are compiled in parallel and linked into `selectivenet_for_semantic_segmentation_binary_amd/libselunet.so`,
next to this file, so the built library travels with the repository snapshot to the GPU box.

Rebuilds are decided by content, not timestamps: each object carries a stamp holding the SHA-256 of
its source, every header and the compiler flags, and the library embeds the fingerprint of the whole
source set (`selunet_build_id()`), which `_lib.load()` compares with the sources next to it — a
library built from other sources than the tree it is loaded from is refused.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libselunet.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "selunet.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SELUNET_ARCH", "gfx950")
# the source fingerprint covers these flags; the target arch (SELUNET_ARCH, default gfx950) is recorded
# beside it in the build id, so a library built for another arch is reported as such, not as stale sources
BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
              "-Wno-unused-but-set-variable"]
FLAGS = BASE_FLAGS + [f"--offload-arch={ARCH}"]


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    return hs + [HEADER]


def _digest(paths, extra=()):
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    for e in extra:
        h.update(e.encode() + b"\0")
    return h.hexdigest()


def source_fingerprint() -> str:
    """SHA-256 (first 24 hex digits) over every kernel source, header and the compiler flags (not the
    target arch: see build_id)."""
    return _digest([os.path.join(CSRC, s) for s in _sources()] + _headers(), BASE_FLAGS)[:24]


def build_id(fp: str | None = None, arch: str | None = None) -> str:
    """The string `selunet_build_id()` returns: '<source fingerprint> <arch>'."""
    return f"{fp or source_fingerprint()} {arch or ARCH}"


def parse_build_id(bid: str) -> tuple[str, str]:
    fp, _, arch = bid.strip().partition(" ")
    return fp, arch or "?"


def lib_stamp_fingerprint(lib: str = None) -> str | None:
    """Source fingerprint recorded next to a built library (its .sha stamp), or None."""
    bid = lib_stamp(lib)
    return parse_build_id(bid)[0] if bid else None


def lib_stamp(lib: str = None) -> str | None:
    """The full build id ('<fingerprint> <arch>') recorded next to a built library, or None."""
    try:
        with open((lib or LIB) + ".sha") as f:
            return f.read().strip()
    except OSError:
        return None


def _stamp_ok(stamp, want):
    try:
        with open(stamp) as f:
            return f.read().strip() == want
    except OSError:
        return False


def _compile(path, obj, want, force):
    stamp = obj + ".sha"
    if not force and os.path.exists(obj) and _stamp_ok(stamp, want):
        return obj
    tmp = f"{obj}.{os.getpid()}.tmp"
    cmd = [HIPCC, *FLAGS, "-c", path, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(path)}:\n{r.stderr[-6000:]}")
    os.replace(tmp, obj)
    with open(stamp, "w") as f:
        f.write(want)
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile and link under an exclusive file lock (several ranks of one node may call it at once
    through load(auto_build=True): the first builds, the others wait and find the stamp current); the
    library is linked to a temporary path and renamed into place, so a process that already mapped the
    old file keeps a consistent image."""
    import fcntl
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(force, verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(force, verbose):
    srcs = _sources()
    heads = _headers()
    fp = build_id()
    # the build id: a one-line translation unit generated from the fingerprint and the arch
    bid_src = os.path.join(BUILD, "build_id.hip")
    bid = f'extern "C" const char* selunet_build_id(void) {{ return "{fp}"; }}\n'
    if not os.path.exists(bid_src) or open(bid_src).read() != bid:
        with open(bid_src, "w") as f:
            f.write(bid)
    jobs = [(os.path.join(CSRC, s), os.path.join(BUILD, s.replace(".hip", ".o")),
             _digest([os.path.join(CSRC, s)] + heads, FLAGS)) for s in srcs]
    jobs.append((bid_src, os.path.join(BUILD, "build_id.o"), _digest([bid_src], FLAGS)))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        objs = list(ex.map(lambda j: _compile(*j, force), jobs))
    lib_stamp = LIB + ".sha"
    if force or not os.path.exists(LIB) or not _stamp_ok(lib_stamp, fp):
        tmp = f"{LIB}.{os.getpid()}.tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, LIB)
        with open(lib_stamp, "w") as f:
            f.write(fp)
    if verbose:
        print(f"built {LIB} (sources {fp})")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
