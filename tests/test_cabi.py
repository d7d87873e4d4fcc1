"""The C-ABI boundary (include/selunet.h) without a GPU.

* every function the header declares is exported by libselunet.so and bound in `_lib.SIGNATURES`
  (and nothing is bound that the header does not declare);
* the ctypes mirrors of the header's structs have the C compiler's size and field offsets
  (a small C program built with gcc against the header prints them);
* the host-only entry points answer without touching a device (version, size queries,
  argument validation with a readable `selunet_last_error`);
* the product path refuses to run without the library (no CPU fallback).
"""
import ctypes
import os
import re
import subprocess

import pytest

from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from selectivenet_for_semantic_segmentation_binary_amd import build as B

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "selunet.h")


def _declared():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(selunet_[A-Za-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(K.lib_path()):
        B.build()
    return ctypes.CDLL(K.lib_path())


def test_header_declarations_are_exported_and_bound(lib):
    decl = _declared()
    assert len(decl) >= 30, decl
    missing = [f for f in decl if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(K.SIGNATURES) == decl


STRUCTS = {
    "selunet_source": (K.Source, ["data", "scale", "shift", "channels", "relu", "layout", "reserved"]),
    "selunet_gather": (K.Gather, ["n", "h", "w", "taps", "nsrc", "reserved", "src"]),
    "selunet_epilogue": (K.Epilogue, ["out0", "out1", "bias", "stats", "mode", "split", "colsum", "bnb"]),
    "selunet_bn_bwd_stats": (K.BnBwdStats, ["y", "scale", "shift", "mean", "invstd", "slab"]),
    "selunet_adam_tensor": (K.AdamTensor, ["param", "grad", "exp_avg", "exp_avg_sq", "numel", "chunk_begin"]),
}


def test_struct_layouts_match_the_c_compiler(tmp_path):
    src = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for s, (_, fields) in STRUCTS.items():
        src.append(f'printf("{s} size %zu\\n", sizeof({s}));')
        for f in fields:
            src.append(f'printf("{s} {f} %zu\\n", offsetof({s}, {f}));')
    src.append('printf("consts %d %d %d\\n", SELUNET_GEMM_BM, SELUNET_ADAM_CHUNK, SELUNET_EP_SCATTER2X);')
    src.append("return 0;}")
    c = tmp_path / "abi.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(line.split()[:2]): int(line.split()[2]) for line in out if line and not line.startswith("consts")}
    for s, (cls, fields) in STRUCTS.items():
        assert got[(s, "size")] == ctypes.sizeof(cls), s
        for f in fields:
            assert got[(s, f)] == getattr(cls, f).offset, (s, f)
    consts = [line for line in out if line.startswith("consts")][0].split()[1:]
    assert list(map(int, consts)) == [K.GEMM_BM, K.ADAM_CHUNK, K.EP_SCATTER2X]


def test_host_queries_need_no_device(lib):
    h = K.load()
    assert h.selunet_version() >= 1
    assert K.query("selunet_channel_slab_rows", 1 << 20) > 0
    assert K.query("selunet_loss_slab_rows", 1 << 20) > 0
    assert K.query("selunet_reduce_ws_bytes", 4) > 0
    assert K.query("selunet_wgrad_ld", 9 * 64) >= 9 * 64
    import torch
    fake = torch.empty(64, dtype=torch.bfloat16)  # never dereferenced: the query inspects shapes/alignment
    g = K.gather(2, 32, 32, 9, K.source(fake, 64))
    assert K.query("selunet_gemm_stats_rows", ctypes.byref(g), 64, K.BF16) in (2 * 2 * 2, 2 * 32 * 32 // K.GEMM_BM)
    g = K.gather(2, 8, 8, 1, K.source(fake, 64))  # 1x1 taps: generic kernel, one stats row per 128 pixels
    assert K.query("selunet_gemm_stats_rows", ctypes.byref(g), 64, K.BF16) == 1
    assert K.query("selunet_gemm_kernel_name", ctypes.byref(g), None, 64, K.EP_PLAIN, K.BF16) == b"gemm_gather<bf16>"
    # split-fp16 3x3 conv, 64 columns: the option SELUNET_OPT_X2D picks the kernel and its slab rows
    f32 = torch.empty(64, dtype=torch.float32)
    scale = torch.ones(64)
    fwd = K.gather(4, 64, 64, 9, K.source(f32, 64, scale, scale))  # BN+ReLU source: a forward
    dgr = K.gather(4, 64, 64, 9, K.source(f32, 64))
    name = lambda g: K.query("selunet_conv3x3_x2_kernel_name", ctypes.byref(g), 64, K.EP_PLAIN, 0)  # noqa: E731
    rows = lambda g: K.query("selunet_conv3x3_x2_stats_rows", ctypes.byref(g), 64)  # noqa: E731
    prev = K.set_option("X2D", -1)
    try:
        assert name(fwd) == b"conv3x3_x2d<f32,64>" and rows(fwd) == 4 * 4 * 4  # one row per 16x16 tile
        assert name(dgr) == b"conv3x3_x2<f32,64>"
        K.set_option("X2D", 0)
        assert name(fwd) == b"conv3x3_x2<f32,64>"
        K.set_option("X2D", 1)
        assert name(dgr) == b"conv3x3_x2d<f32,64>"
    finally:
        K.set_option("X2D", prev)


def test_invalid_arguments_fail_with_a_message(lib):
    h = K.load()
    # unsupported channel count for the BN reduction: rejected on the host before any launch
    rc = h.selunet_channel_sum(None, 10, 3, None, K.F32, None)
    assert rc == 1
    assert h.selunet_last_error()
    with pytest.raises(RuntimeError):
        K.call("selunet_channel_sum", None, 10, 3, None, K.F32, None)


def test_product_path_has_no_cpu_fallback():
    import torch

    import selectivenet_for_semantic_segmentation_binary_amd as S
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    net = S.UNet_B("RGB", selective=True)
    with pytest.raises(RuntimeError):
        net(torch.zeros(1, 3, 16, 16))
    with pytest.raises(RuntimeError):
        S.calc_selective_risk_image_b(torch.zeros(1, 4, 4), torch.zeros(1, 4, 4), torch.zeros(1, 4, 4))


def test_build_id_carries_the_sources_and_the_arch(lib, tmp_path):
    """the library's build id is '<source fingerprint> <arch>'; the fingerprint leaves the
    target arch out (a library built for another SELUNET_ARCH is reported as such), and the .sha stamp
    next to the library is what load(auto_build=True) compares before mapping it (stale -> rebuild)."""
    lib.selunet_build_id.restype = ctypes.c_char_p
    fp, arch = B.parse_build_id(lib.selunet_build_id().decode())
    assert fp == B.source_fingerprint() and arch == B.ARCH
    assert B.lib_stamp_fingerprint(K.lib_path()) == fp
    stamp = tmp_path / "x.so.sha"
    stamp.write_text("0123abcd gfx942")
    assert B.lib_stamp_fingerprint(str(tmp_path / "x.so")) == "0123abcd"
    assert B.lib_stamp_fingerprint(str(tmp_path / "missing.so")) is None
    assert not any("offload-arch" in f for f in B.BASE_FLAGS)
