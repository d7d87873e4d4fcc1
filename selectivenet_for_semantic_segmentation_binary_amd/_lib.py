"""ctypes binding of libselunet.so (the C-ABI declared in include/selunet.h).

The product path has no CPU fallback: if the library is missing or cannot be
loaded, every entry point raises. Build it with
``python -m selectivenet_for_semantic_segmentation_binary_amd.build``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import build as _build

c_int32, c_int64, c_double, c_float, c_void_p = (ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                                                ctypes.c_float, ctypes.c_void_p)

F32, BF16 = 0, 1
EP_PLAIN, EP_SPLIT, EP_SCATTER2X = 0, 1, 2
DA_TENSOR, DA_POOL, DA_HEADS = 0, 1, 2  # selunet_da_source kinds
GEMM_BM = 128
ADAM_CHUNK = 4096


class Source(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("scale", c_void_p), ("shift", c_void_p), ("channels", c_int32),
                ("relu", c_int32), ("layout", c_int32), ("reserved", c_int32)]


class Gather(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("taps", c_int32), ("nsrc", c_int32),
                ("reserved", c_int32), ("src", Source * 2)]


class BnBwdStats(ctypes.Structure):
    _fields_ = [("y", c_void_p), ("scale", c_void_p), ("shift", c_void_p), ("mean", c_void_p),
                ("invstd", c_void_p), ("slab", c_void_p), ("amax", c_void_p)]


class DaSource(ctypes.Structure):
    """selunet_da_source: where the fused weight gradient's staging forms dA (SELUNET_DA_*)."""
    _fields_ = [("kind", c_int32), ("nh", c_int32), ("pooled", c_void_p), ("skip", c_void_p), ("head_w", c_void_p),
                ("g", c_void_p * 3)]


class Epilogue(ctypes.Structure):
    _fields_ = [("out0", c_void_p), ("out1", c_void_p), ("bias", c_void_p), ("stats", c_void_p),
                ("mode", c_int32), ("split", c_int32), ("colsum", c_void_p), ("bnb", BnBwdStats),
                ("amax", c_void_p), ("stats_center", c_void_p)]


class PackDesc(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("fwd", c_void_p), ("dgrad", c_void_p), ("kind", c_int32), ("co", c_int32),
                ("ci", c_int32), ("k_pad", c_int32), ("offset", c_int64)]


PACK_MAX, PACK_CONV3X3, PACK_CONVT, PACK_CONV3X3_WINO, PACK_CONV3X3_X2, PACK_CONVT_X2, PACK_COPY = 32, 0, 1, 2, 3, 4, 5
WG_CONV3X3, WG_CONVT = 1, 2  # selunet_gemm_wgrad_ws_to layouts


class PackList(ctypes.Structure):
    _fields_ = [("n", c_int32), ("_pad", c_int32), ("d", PackDesc * PACK_MAX)]


class HeadPlanes(ctypes.Structure):
    _fields_ = [("n", c_int32), ("hw", c_int32), ("plane", c_void_p * 8), ("img_stride", c_int64 * 8),
                ("w_off", c_int32 * 8), ("b_off", c_int32 * 8), ("row_len", c_int32)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", c_int64), ("chunk_begin", c_int64)]


P = c_void_p
# name -> (restype, argtypes); mirrors include/selunet.h
SIGNATURES = {
    "selunet_last_error": (ctypes.c_char_p, []),
    "selunet_version": (c_int32, []),
    "selunet_build_id": (ctypes.c_char_p, []),
    "selunet_pack_conv3x3": (c_int32, [P, c_int32, c_int32, c_int32, P, P, c_int32, P]),
    "selunet_pack_convT": (c_int32, [P, c_int32, c_int32, P, P, c_int32, P]),
    "selunet_unpack_conv3x3_grad": (c_int32, [P, c_int32, c_int32, c_int32, P, P]),
    "selunet_unpack_convT_grad": (c_int32, [P, c_int32, c_int32, P, P]),
    "selunet_gemm_gather": (c_int32, [ctypes.POINTER(Gather), P, c_int32, c_int32, ctypes.POINTER(Epilogue),
                                      c_int32, P]),
    "selunet_gemm_wgrad": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, c_int32, P]),
    "selunet_wgrad_ld": (c_int32, [c_int32]),
    "selunet_gemm_wgrad_ws_bytes": (c_int64, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), c_int32]),
    "selunet_gemm_wgrad_ws": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, P, c_int64, c_int32, P]),
    "selunet_gemm_wgrad_ws_to": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, P, c_int64, c_int32, P,
                                           c_int32, P]),
    "selunet_conv3x3_wino_ok": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "selunet_conv3x3_wino": (c_int32, [ctypes.POINTER(Gather), P, c_int32, ctypes.POINTER(Epilogue), P]),
    "selunet_conv3x3_wino_kernel_name": (ctypes.c_char_p, [c_int32, c_int32, c_int32]),
    "selunet_conv3x3_x2_ok": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "selunet_gemm_gather_x2": (c_int32, [ctypes.POINTER(Gather), P, c_int32, c_int32, ctypes.POINTER(Epilogue), P, P,
                                         P]),
    "selunet_conv3x3_x2": (c_int32, [ctypes.POINTER(Gather), P, c_int32, ctypes.POINTER(Epilogue), P, P, P]),
    "selunet_conv3x3_x2_kernel_name": (ctypes.c_char_p, [ctypes.POINTER(Gather), c_int32, c_int32, c_int32]),
    "selunet_conv3x3_x2_stats_rows": (c_int64, [ctypes.POINTER(Gather), c_int32]),
    "selunet_act_bound": (c_int32, [P, P, c_int32, c_int64, P, P]),
    "selunet_conv3x3_wgrad_x2_ws_bytes": (c_int64, [ctypes.POINTER(Gather), ctypes.POINTER(Gather)]),
    "selunet_gemm_wgrad_x2_ws_bytes": (c_int64, [ctypes.POINTER(Gather), ctypes.POINTER(Gather)]),
    "selunet_gemm_wgrad_x2": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, c_int64, c_int32, P, P, P,
                                        P, P, P]),
    "selunet_conv3x3_wgrad_x2": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, c_int64, P, P, P, P,
                                           P]),
    "selunet_conv3x3_wgrad_x2_bn": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, c_int64, P, P, P, P,
                                              ctypes.POINTER(BnBwdStats), P, P, P, P]),
    "selunet_conv3x3_wgrad_x2_bn_src": (c_int32, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), P, c_int64, P, P, P,
                                                  P, ctypes.POINTER(BnBwdStats), P, ctypes.POINTER(DaSource), P, P,
                                                  P]),
    "selunet_gemm_stats_rows": (c_int64, [ctypes.POINTER(Gather), c_int32, c_int32]),
    "selunet_gemm_gather_x2_stats_rows": (c_int64, [ctypes.POINTER(Gather), c_int32]),
    "selunet_set_halo_workgroups": (c_int32, [c_int32]),
    "selunet_set_gather_workgroups": (c_int32, [c_int32]),
    "selunet_gemm_kernel_name": (ctypes.c_char_p, [ctypes.POINTER(Gather), ctypes.POINTER(Gather), c_int32, c_int32,
                                                   c_int32]),
    "selunet_reduce_ws_bytes": (c_int64, [c_int32]),
    "selunet_reduce_rows": (c_int32, [P, c_int64, c_int32, P, P, P, P]),
    "selunet_channel_slab_rows": (c_int64, [c_int64]),
    "selunet_bn_centered_rows": (c_int64, [c_int64]),
    "selunet_channel_sum": (c_int32, [P, c_int64, c_int32, P, c_int32, P]),
    "selunet_bn_finalize": (c_int32, [P, c_int64, c_int32, P, P, P, P, P, P, c_float, c_float, c_int32, P, P, P, P,
                                      P]),
    "selunet_bn_bwd_reduce": (c_int32, [P, P, c_int64, c_int32, P, P, P, P, P, c_int32, P]),
    "selunet_bn_bwd_finalize": (c_int32, [P, c_int64, c_int32, P, P, P, P, P, P, P]),
    "selunet_pack_weights": (c_int32, [ctypes.POINTER(PackList), c_int32, P]),
    "selunet_bn_stats_finalize": (c_int32, [P, c_int64, P, P, c_int64, c_int32, P, P, P, P, P, P, c_float, c_float,
                                            P, P, P, P, P]),
    "selunet_bn_centered_partials": (c_int32, [P, c_int64, c_int32, P, P, c_int32, P]),
    "selunet_bn_centered_partials_adaptive": (c_int32, [P, c_int64, c_int32, P, P, c_float, P, c_int32, P]),
    "selunet_bn_stats_finalize_centered": (c_int32, [P, c_int64, P, P, c_int64, c_int32, P, P, P, P, P, P, P,
                                                     c_float, c_float, P, P, P, P, P]),
    "selunet_bn_stats_finalize_centered_bound": (c_int32, [P, c_int64, P, P, c_int64, c_int32, P, P, P, P, P, P, P,
                                                           c_float, c_float, P, P, P, P, P, P]),
    "selunet_bn_bwd_stats_finalize": (c_int32, [P, c_int64, P, P, c_int64, c_int32, P, P, P, P, P, P, P]),
    "selunet_bn_bwd_stats_finalize_bound": (c_int32, [P, c_int64, P, P, c_int64, c_int32, P, P, P, P, P, P, P, P, P]),
    "selunet_bn_bwd_apply": (c_int32, [P, P, c_int64, c_int32, P, P, P, P, P, P, c_int32, P]),
    "selunet_bn_bwd_apply_amax": (c_int32, [P, P, c_int64, c_int32, P, P, P, P, P, P, P, c_int32, P]),
    "selunet_bn_bwd_apply_heads": (c_int32, [P, c_int64, P, P, P, P, P, P, c_int32, P, P, P, P, P, c_int32, P]),
    "selunet_bn_bwd_apply_heads_planes": (c_int32, [P, c_int64, P, P, P, P, P, P, ctypes.POINTER(HeadPlanes), P, P,
                                                    c_int32, P]),
    "selunet_bn_bwd_apply_pool": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, P, P, P, P, P, P,
                                            c_int32, P]),
    "selunet_im2col3x3": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, c_int32, P, c_int32, P]),
    "selunet_maxpool2_fwd": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, c_int32, P]),
    "selunet_maxpool2_bwd": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, P, P,
                                       ctypes.POINTER(BnBwdStats), c_int32, P]),
    "selunet_maxpool2_bwd_slab_rows": (c_int64, [c_int32, c_int32, c_int32, c_int32]),
    "selunet_first_conv_rows": (c_int64, [c_int32, c_int32, c_int32]),
    "selunet_first_conv_fwd": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, c_int32, P]),
    "selunet_first_conv_fwd_centered": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, P, c_int32, P]),
    "selunet_bn_stats_finalize_shifted": (c_int32, [P, c_int64, P, c_int64, c_int32, P, P, P, P, c_float, P, P, P, P,
                                                    P, P]),
    "selunet_first_conv_wgrad_rows": (c_int64, [c_int32, c_int32, c_int32]),
    "selunet_first_conv_wgrad": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, c_int32, P]),
    "selunet_first_conv_wgrad_bn": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, P, P, P, P, P, c_int32,
                                              P]),
    "selunet_heads_fwd": (c_int32, [P, c_int64, P, P, P, P, c_int32, P, P, P, c_int32, P]),
    "selunet_heads_bwd": (c_int32, [P, c_int64, P, P, P, c_int32, P, P, P, P, P, ctypes.POINTER(BnBwdStats),
                                    c_int32, P]),
    "selunet_heads_fwd_planes": (c_int32, [P, c_int64, P, P, P, P, ctypes.POINTER(HeadPlanes), c_int32, P]),
    "selunet_heads_bwd_planes": (c_int32, [P, c_int64, P, P, P, ctypes.POINTER(HeadPlanes), P, P,
                                           ctypes.POINTER(BnBwdStats), c_int32, P]),
    "selunet_ce_selective_partials": (c_int32, [P, P, P, c_int64, c_int32, c_int64, P, P]),
    "selunet_ce_selective_bwd": (c_int32, [P, P, P, c_int64, c_int32, c_int64, P, c_float, P, P, P, P, P]),
    "selunet_ce_selective_partials_hard": (c_int32, [P, P, P, c_int64, c_int32, c_int64, P, P]),
    "selunet_ce_selective_bwd_hard": (c_int32, [P, P, P, c_int64, c_int32, c_int64, P, P, P, P, P]),
    "selunet_ce_partials": (c_int32, [P, P, c_int64, c_int32, c_int64, P, P]),
    "selunet_ce_bwd": (c_int32, [P, P, c_int64, c_int32, c_int64, c_double, P, P, P]),
    "selunet_loss_slab_rows": (c_int64, [c_int64]),
    "selunet_selective_partials": (c_int32, [P, P, P, c_int64, P, P]),
    "selunet_selective_finalize": (c_int32, [P, c_double, c_float, c_float, P, P, P, P]),
    "selunet_selective_bwd": (c_int32, [P, P, P, c_int64, P, c_float, P, P, P, P, P]),
    "selunet_selective_partials_hard": (c_int32, [P, P, P, c_int64, P, P]),
    "selunet_selective_bwd_hard": (c_int32, [P, P, P, c_int64, P, P, P, P, P]),
    "selunet_bce_partials": (c_int32, [P, P, c_int64, P, P]),
    "selunet_bce_finalize": (c_int32, [P, c_double, P, P]),
    "selunet_bce_bwd": (c_int32, [P, P, c_int64, c_double, P, P, P]),
    "selunet_adam_step": (c_int32, [P, c_int32, c_int64, c_float, c_float, c_float, c_float, c_float, c_int64, P]),
    "selunet_memset": (c_int32, [P, c_int32, c_int64, P]),
    "selunet_memcpy": (c_int32, [P, P, c_int64, P]),
    "selunet_stream_create": (c_int32, [ctypes.POINTER(P)]),
    "selunet_stream_destroy": (c_int32, [P]),
    "selunet_graph_capture_begin": (c_int32, [P]),
    "selunet_graph_capture_end": (c_int32, [P, ctypes.POINTER(P)]),
    "selunet_graph_launch": (c_int32, [P, P]),
    "selunet_graph_destroy": (c_int32, [P]),
    "selunet_prep_batch": (c_int32, [P, P, P, c_int32, c_int32, c_int32, c_int32, P, P, P]),
    "selunet_prep_batch_mode": (c_int32, [P, P, P, c_int32, c_int32, c_int32, c_int32, P, P, P]),
    "selunet_seg_metrics": (c_int32, [P, P, P, c_int64, c_float, c_float, P, P]),
    "selunet_set_option": (c_int64, [c_int32, c_int64]),
    "selunet_cu_hold": (c_int32, [P, P, c_int64, c_int32, c_float, P]),
}

_lib = None
_lock = threading.Lock()


def lib_path() -> str:
    """The in-tree build; SELUNET_LIB overrides it (A/B timing of kernel variants)."""
    return os.environ.get("SELUNET_LIB", _build.LIB)


def load(auto_build: bool = False):
    """Load (optionally build) libselunet.so; raise RuntimeError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        tree = _build.source_fingerprint()
        own = "SELUNET_LIB" not in os.environ
        if auto_build and own and (not os.path.exists(path) or _build.lib_stamp(path) != _build.build_id(tree)):
            # missing, stale or built for another arch: rebuild before the library is mapped (build() holds a
            # file lock, so the ranks of one node build once)
            _build.build(verbose=False)
        if not os.path.exists(path):
            raise RuntimeError(
                f"{path} not found: the MI355X kernels are not built (run "
                "`python -m selectivenet_for_semantic_segmentation_binary_amd.build`). "
                "There is no CPU fallback.")
        L = ctypes.CDLL(path)
        L.selunet_build_id.restype = ctypes.c_char_p
        built_fp, built_arch = _build.parse_build_id(L.selunet_build_id().decode())
        if own and built_fp != tree:
            raise RuntimeError(
                f"{path} was built from other sources (build id {built_fp}, for {built_arch}; tree "
                f"{tree}): rebuild with `python -m selectivenet_for_semantic_segmentation_binary_amd.build`")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        for env, key in ENV_OPTIONS.items():  # the host's choices; the library reads no environment
            v = os.environ.get(env)
            if v is not None and v.strip().lstrip("-").isdigit():
                L.selunet_set_option(key, int(v))
        if os.environ.get("SELUNET_NO_HALO") == "1":
            L.selunet_set_option(OPT["HALO"], 0)
    return _lib


# selunet_option keys (include/selunet.h)
OPT = {name: i for i, name in enumerate([
    "HALO", "HALO_PERSIST", "WINO", "WINO_WGRAD", "WINO_WGRAD_TW", "WINO_WGRAD_WAVES", "WGRAD_WGS",
    "X2_WGRAD_WGS", "GEMM_WGRAD_WGS", "GATHER_WGS", "RF_SINGLE", "APPLY_U8", "APPLY_GRID", "X2D",
    "TILE_QUEUE", "X2P", "CONVT_RING"])}
# environment variables the host maps onto options at load (A/B and ablation runs of tools/ and the
# exact-fp32 comparison paths of the tests); SELUNET_NO_HALO=1 means HALO=0
ENV_OPTIONS = {f"SELUNET_{k}": v for k, v in OPT.items() if k != "HALO"}


def set_option(name: str, value: int) -> int:
    """selunet_set_option by name (OPT); value < 0 restores the default. Returns the previous value."""
    return int(load().selunet_set_option(OPT[name], int(value)))


class SelunetError(RuntimeError):
    pass


_HOOK = None


def set_call_hook(hook):
    """Install hook(name, args, fn) -> rc around every entry-point call (profiling), None to clear."""
    global _HOOK
    _HOOK = hook


def call(name, *args):
    L = load()
    fn = getattr(L, name)
    if _REC is not None:
        _REC.record(name, fn, args)
    rc = fn(*args) if _HOOK is None else _HOOK(name, args, lambda: fn(*args))
    if rc != 0:
        raise SelunetError(f"{name}: {L.selunet_last_error().decode()}")
    return rc


# ----------------------------------------------------------------------------- launch plans
class Slot:
    """A recorded pointer argument that points into a per-call buffer: rebound at replay."""
    __slots__ = ("name", "offset")

    def __init__(self, name, offset):
        self.name, self.offset = name, offset


class Plan:
    """The exact sequence of C-ABI calls one engine pass made, with their (already converted)
    arguments. Replaying it re-issues the same launches without re-running the Python sequencing
    (allocation, descriptor building, queries): the host cost of a step drops to the ctypes calls.
    Pointer arguments that fall inside a registered per-call buffer (the network input, the head
    outputs, the incoming head gradients, the gradient buffer) are recorded as Slots and rebound
    to that call's buffers; every other pointer refers to memory the plan owns."""

    MAX_GRAPHS = 4  # captured graphs kept per plan (one per set of per-call buffer addresses)

    def __init__(self, slots):
        self._ranges = [(n, t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for n, t in slots.items()
                        if t is not None]
        self.calls = []  # (name, fn, args, slot_positions)
        self.keep = []   # every buffer the recorded calls touch stays allocated for the plan's life
        self.stream = stream_ptr()  # every recorded launch's last argument (engine signatures key on it)
        self._graphs = {}   # per-call buffer addresses -> [graph exec or ("marker", tag)], LRU order
        self._seen = set()
        self._graphable = graphs_enabled()

    def _slot(self, v):
        if isinstance(v, int) and v:
            for n, lo, hi in self._ranges:
                if lo <= v < hi:
                    return Slot(n, v - lo)
        return None

    def record(self, name, fn, args):
        args = list(args)
        pos = []
        for i, a in enumerate(args):
            if isinstance(a, ctypes.Structure):
                fields = _struct_slots(a, self._slot)
                if fields:  # per-call buffers inside a descriptor: rebound in a copy at replay
                    args[i] = _StructSlots(type(a).from_buffer_copy(a), fields)
                    pos.append(i)
                continue
            sl = self._slot(a)
            if sl is not None:
                args[i] = sl
                pos.append(i)
        self.calls.append((name, fn, tuple(args), tuple(pos)))

    def record_marker(self, tag):
        self.calls.append((None, None, tag, ()))

    def _bound(self, base):
        """(name, fn, args) of every recorded call with its per-call buffers rebound; markers as
        (None, None, tag)."""
        for name, fn, args, pos in self.calls:
            if pos:
                a = list(args)
                for i in pos:
                    a[i] = a[i].bind(base) if isinstance(a[i], _StructSlots) else base[a[i].name] + a[i].offset
                args = a
            yield name, fn, args

    def replay(self, slots, on_marker=None):
        """Re-issue the recorded launches for this call's buffers. The second time a set of buffer
        addresses is seen (a training loop's steady state: the caching allocator hands the same
        blocks back), the launches between markers are captured into HIP graphs; from then on a
        replay is one selunet_graph_launch per segment plus the host-side marker hooks."""
        base = {n: t.data_ptr() for n, t in slots.items() if t is not None}
        L = load()
        if self._graphable and _HOOK is None and _REC is None:
            key = tuple(sorted(base.items()))
            segs = self._graphs.pop(key, None)
            if segs is None and key in self._seen:
                segs = self._capture(base, L)
            if len(self._seen) > 64:  # addresses that never repeat: stay on per-launch replay
                self._seen.clear()
            self._seen.add(key)
            if segs is not None:
                self._graphs[key] = segs  # most recently used last
                while len(self._graphs) > self.MAX_GRAPHS:
                    _destroy_graphs(self._graphs.pop(next(iter(self._graphs))))
                stream = self.stream
                for s in segs:
                    if isinstance(s, tuple):
                        if on_marker is not None:
                            on_marker(s[1])
                    elif L.selunet_graph_launch(s, stream) != 0:
                        raise SelunetError(f"selunet_graph_launch: {L.selunet_last_error().decode()}")
                return
        for name, fn, args in self._bound(base):
            if name is None:  # marker: host-side hook between launches (e.g. a gradient bucket's all-reduce)
                if on_marker is not None:
                    on_marker(args)
                continue
            rc = fn(*args) if _HOOK is None else _HOOK(name, args, lambda fn=fn, args=args: fn(*args))
            if rc != 0:
                raise SelunetError(f"{name}: {L.selunet_last_error().decode()}")

    def _capture(self, base, L):
        """Capture the plan's launches (segments between markers) on the private capture stream;
        None (and the plan stays on per-launch replay) if the capture fails."""
        cap = capture_stream()
        segs, open_ = [], False

        def close():
            ex = ctypes.c_void_p()
            if L.selunet_graph_capture_end(cap, ctypes.byref(ex)) != 0:
                raise SelunetError(f"selunet_graph_capture_end: {L.selunet_last_error().decode()}")
            segs.append(ex.value)

        try:
            for name, fn, args in self._bound(base):
                if name is None:
                    if open_:
                        close()
                        open_ = False
                    segs.append(("marker", args))
                    continue
                if args[-1] != self.stream and not (args[-1] is None and not self.stream):
                    raise SelunetError(f"{name}: recorded on another stream")
                if not open_:
                    if L.selunet_graph_capture_begin(cap) != 0:
                        raise SelunetError(f"selunet_graph_capture_begin: {L.selunet_last_error().decode()}")
                    open_ = True
                if fn(*args[:-1], cap) != 0:
                    raise SelunetError(f"{name} (capture): {L.selunet_last_error().decode()}")
            if open_:
                close()
                open_ = False
        except SelunetError:
            if open_:
                ex = ctypes.c_void_p()
                L.selunet_graph_capture_end(cap, ctypes.byref(ex))
                L.selunet_graph_destroy(ex.value)
            _destroy_graphs(segs)
            self._graphable = False
            return None
        return segs

    def __del__(self):
        try:
            for segs in self._graphs.values():
                _destroy_graphs(segs)
            self._graphs = {}
        except Exception:  # interpreter shutdown
            pass


def fused_apply_enabled():
    """BN-backward apply forming dA on the fly for the heads / max-pool producers
    (selunet_bn_bwd_apply_heads / _pool, the producers in sums-only mode). SELUNET_FUSED_APPLY=0: the
    unfused kernels (dA written by the producer, read by selunet_bn_bwd_apply), for A/B runs and tests."""
    return os.environ.get("SELUNET_FUSED_APPLY", "1") != "0"


def graphs_enabled():
    """HIP-graph replay of launch plans: opt-in with SELUNET_GRAPHS=1. Measured on MI355X, a
    bs=16 bf16 step is GPU-bound (6.17 ms per-launch replay, 6.26 ms graphs), so it is off by
    default; it removes the per-launch host cost when the host is the contended resource."""
    return os.environ.get("SELUNET_GRAPHS", "0") == "1"


_CAP_STREAMS = {}


def capture_stream():
    """The private non-blocking stream launch plans are captured on (one per device)."""
    dev = torch.cuda.current_device()
    s = _CAP_STREAMS.get(dev)
    if s is None:
        h = ctypes.c_void_p()
        if load().selunet_stream_create(ctypes.byref(h)) != 0:
            raise SelunetError(f"selunet_stream_create: {load().selunet_last_error().decode()}")
        s = _CAP_STREAMS[dev] = h.value
    return s


def _destroy_graphs(segs):
    L = _lib
    if L is None:
        return
    for s in segs:
        if not isinstance(s, tuple) and s:
            L.selunet_graph_destroy(s)


def _struct_slots(st, slot_of, path=()):
    """(field path, Slot) of every pointer field of a (nested) descriptor that points into a
    registered per-call buffer; a path step is a field name or (array field, index)."""
    out = []
    for f, _ in st._fields_:
        v = getattr(st, f)
        if isinstance(v, ctypes.Structure):
            out += _struct_slots(v, slot_of, path + (f,))
        elif isinstance(v, ctypes.Array):
            for i, e in enumerate(v):
                if isinstance(e, ctypes.Structure):
                    out += _struct_slots(e, slot_of, path + ((f, i),))
                else:
                    sl = slot_of(e)
                    if sl is not None:
                        out.append((path + ((f, i),), sl))
        else:
            sl = slot_of(v)
            if sl is not None:
                out.append((path + (f,), sl))
    return out


class _StructSlots:
    """A recorded descriptor whose pointer fields into per-call buffers are rebound per replay."""

    def __init__(self, st, fields):
        self.st, self.fields = st, fields

    def bind(self, base):
        st = type(self.st).from_buffer_copy(self.st)
        for path, sl in self.fields:
            obj = st
            for step in path[:-1]:
                obj = getattr(obj, step[0])[step[1]] if isinstance(step, tuple) else getattr(obj, step)
            last, v = path[-1], base[sl.name] + sl.offset
            if isinstance(last, tuple):
                getattr(obj, last[0])[last[1]] = v
            else:
                setattr(obj, last, v)
        return st


_REC = None


_MARKER_CB = None


def marker(tag):
    """A point in the launch sequence where host code may act (the gradients of a layer are
    enqueued): calls the active marker callback now and, while recording, stores the marker in the
    plan so replays call their callback at the same point."""
    if _REC is not None:
        _REC.record_marker(tag)
    if _MARKER_CB is not None:
        _MARKER_CB(tag)


class marker_callback:
    """Context manager installing the callback `marker` calls during a (recorded) pass."""

    def __init__(self, cb):
        self.cb = cb

    def __enter__(self):
        global _MARKER_CB
        self.prev, _MARKER_CB = _MARKER_CB, self.cb
        return self

    def __exit__(self, *exc):
        global _MARKER_CB
        _MARKER_CB = self.prev
        return False


def keep(t):
    """Allocation made by recorded sequencing: owned by the plan being recorded (if any)."""
    if _REC is not None and t is not None:
        _REC.keep.append(t)
    return t


class recording:
    """Context manager: record every `call` made inside into `plan`."""

    def __init__(self, plan):
        self.plan = plan

    def __enter__(self):
        global _REC
        if _REC is not None:
            raise RuntimeError("nested plan recording")
        _REC = self.plan
        return self.plan

    def __exit__(self, *exc):
        global _REC
        _REC = None
        return False


def query(name, *args):
    return getattr(load(), name)(*args)


# ----------------------------------------------------------------------------- tensor helpers
def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"unsupported activation dtype {dt}")


def source(data, channels, scale=None, shift=None, relu=True, layout=0, amax=None) -> Source:
    """A gather source; amax (a 1-element fp32 device tensor, optional) is the range word of the
    source's values after its transform, kept on the Python object for selunet_conv3x3_x2."""
    s = Source(ptr(data), ptr(scale), ptr(shift), channels, int(bool(relu) and scale is not None), layout, 0)
    s.amax = amax
    return s


def gather(n, h, w, taps, *srcs: Source) -> Gather:
    g = Gather(n, h, w, taps, len(srcs), 0)
    for i, s in enumerate(srcs):
        g.src[i] = s
    return g
