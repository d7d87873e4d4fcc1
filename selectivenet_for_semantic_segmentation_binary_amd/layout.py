"""Static description of the UNet_B graph: layer names, channel counts, parameter
registration order and the seeded initialisation recipe.

Everything here mirrors `model.py` of the reference so that the state_dict keys,
shapes and parameter order (= Adam state indices) are identical:

* `CBR_2D` blocks (`model.py:9-15`): ``<name>.0.weight [Co,Ci,3,3]``,
  ``<name>.0.bias [Co]``, ``<name>.1.weight/bias [Co]`` plus BN buffers
  ``running_mean``, ``running_var``, ``num_batches_tracked``.
* `UNet_B.__init__` registration order (`model.py:19-66`): enc 1_1..3_2,
  bottleneck 4_2/4_1, unpool3, dec 3_2/3_1, unpool2, dec 2_2/2_1, unpool1,
  dec 1_2/1_1, conv1x1, then conv_select / conv_aux when selective.
* `ConvTranspose2d(k=2, s=2)` weights are ``[Ci, Co, 2, 2]`` (`model.py:44,51,57`).

The init recipe is numpy-PCG64 seeded so the same weights can be produced in
this container (to drive the reference when generating golden fixtures) and on
the GPU box (where the reference never travels).
"""
from __future__ import annotations

import numpy as np

# (name, C_in, C_out) of every CBR_2D block, in forward order (model.py:29-61).
# C_in of encoder_layer_1_1 depends on input_type (model.py:24-27).
CBR_LAYERS = [
    ("encoder_layer_1_1", None, 64),
    ("encoder_layer_1_2", 64, 64),
    ("encoder_layer_2_1", 64, 128),
    ("encoder_layer_2_2", 128, 128),
    ("encoder_layer_3_1", 128, 256),
    ("encoder_layer_3_2", 256, 256),
    ("decoder_layer_4_2", 256, 512),
    ("decoder_layer_4_1", 512, 512),
    ("decoder_layer_3_2", 512, 256),
    ("decoder_layer_3_1", 256, 256),
    ("decoder_layer_2_2", 256, 128),
    ("decoder_layer_2_1", 128, 128),
    ("decoder_layer_1_2", 128, 64),
    ("decoder_layer_1_1", 64, 64),
]

# (name, C_in, C_out) of the ConvTranspose2d(k2,s2) up-samplers (model.py:44,51,57).
UNPOOLS = [("unpool3", 512, 256), ("unpool2", 256, 128), ("unpool1", 128, 64)]

HEADS = ["conv1x1", "conv_select", "conv_aux"]  # model.py:62,65,66


def input_channels(input_type: str) -> int:
    """`model.py:24-27`: 'RGB' anywhere in the string -> 3, exactly 'GH' -> 2."""
    if "RGB" in input_type:
        return 3
    if input_type == "GH":
        return 2
    # The reference leaves input_ch unbound here and fails with UnboundLocalError.
    raise ValueError(f"unsupported input_type {input_type!r} (reference accepts '*RGB*' or 'GH')")


def head_channels(selective: bool, n_cls: int | None = None):
    """[(head, output channels)] in registration order: UNet_B (n_cls None, model.py:62,65-66) has
    1-channel heads; the CE UNet (model.py:170,174-175) conv1x1 -> n_cls, conv_select -> 2,
    conv_aux -> n_cls."""
    if n_cls is None:
        ch = [1, 1, 1]
    else:
        ch = [n_cls, 2, n_cls]
    heads = list(zip(HEADS, ch))
    return heads if selective else heads[:1]


def param_specs(input_type: str = "RGB", selective: bool = False, n_cls: int | None = None):
    """Parameters in registration order: list of (key, shape, kind, fan_in). n_cls: None for
    UNet_B, the class count for the CE `UNet` (model.py:106-191; only the heads differ).

    kind in {conv_w, conv_b, bn_w, bn_b, convT_w, convT_b, head_w, head_b}.
    fan_in follows torch.nn.init._calculate_fan_in_and_fan_out (dim 1 * k*k),
    which is what the reference's default init uses.
    """
    cin0 = input_channels(input_type)
    specs = []

    def cbr(name, ci, co):
        specs.append((f"{name}.0.weight", (co, ci, 3, 3), "conv_w", ci * 9))
        specs.append((f"{name}.0.bias", (co,), "conv_b", ci * 9))
        specs.append((f"{name}.1.weight", (co,), "bn_w", None))
        specs.append((f"{name}.1.bias", (co,), "bn_b", None))

    def unpool(name, ci, co):
        # torch computes fan_in of a ConvTranspose weight [Ci,Co,k,k] from dim 1 = Co.
        specs.append((f"{name}.weight", (ci, co, 2, 2), "convT_w", co * 4))
        specs.append((f"{name}.bias", (co,), "convT_b", co * 4))

    lay = {n: (ci if ci is not None else cin0, co) for n, ci, co in CBR_LAYERS}
    for n in ["encoder_layer_1_1", "encoder_layer_1_2", "encoder_layer_2_1", "encoder_layer_2_2",
              "encoder_layer_3_1", "encoder_layer_3_2", "decoder_layer_4_2", "decoder_layer_4_1"]:
        cbr(n, *lay[n])
    unpool(*UNPOOLS[0])
    cbr("decoder_layer_3_2", *lay["decoder_layer_3_2"])
    cbr("decoder_layer_3_1", *lay["decoder_layer_3_1"])
    unpool(*UNPOOLS[1])
    cbr("decoder_layer_2_2", *lay["decoder_layer_2_2"])
    cbr("decoder_layer_2_1", *lay["decoder_layer_2_1"])
    unpool(*UNPOOLS[2])
    cbr("decoder_layer_1_2", *lay["decoder_layer_1_2"])
    cbr("decoder_layer_1_1", *lay["decoder_layer_1_1"])
    for h, c in head_channels(selective, n_cls):
        specs.append((f"{h}.weight", (c, 64, 1, 1), "head_w", 64))
        specs.append((f"{h}.bias", (c,), "head_b", 64))
    return specs


def buffer_specs():
    """BatchNorm buffers per CBR block, in state_dict order after each block's params."""
    out = []
    for n, _, co in CBR_LAYERS:
        out.append((f"{n}.1.running_mean", (co,)))
        out.append((f"{n}.1.running_var", (co,)))
        out.append((f"{n}.1.num_batches_tracked", ()))
    return out


def state_dict_keys(input_type: str = "RGB", selective: bool = False, n_cls: int | None = None):
    """Exact key order of the reference `UNet_B(...)` / `UNet(...)` `state_dict()`."""
    keys = []
    for key, _, kind, _ in param_specs(input_type, selective, n_cls):
        keys.append(key)
        if kind == "bn_b":
            base = key[: -len(".bias")]
            keys += [f"{base}.running_mean", f"{base}.running_var", f"{base}.num_batches_tracked"]
    return keys


def seeded_params(seed: int = 0, input_type: str = "RGB", selective: bool = False,
                  bn_affine_random: bool = True, n_cls: int | None = None):
    """Deterministic parameter recipe (numpy PCG64), torch-default-like bounds.

    conv/convT/head weights and biases ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (the bound
    torch's kaiming_uniform_(a=sqrt(5)) gives). BN gamma/beta are randomised around
    (1, 0) when `bn_affine_random` so parity tests exercise the affine path.
    Returns an ordered dict key -> float32 ndarray.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for key, shape, kind, fan_in in param_specs(input_type, selective, n_cls):
        if kind in ("bn_w",):
            v = rng.uniform(0.6, 1.4, size=shape) if bn_affine_random else np.ones(shape)
        elif kind in ("bn_b",):
            v = rng.uniform(-0.2, 0.2, size=shape) if bn_affine_random else np.zeros(shape)
        else:
            b = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-b, b, size=shape)
        out[key] = v.astype(np.float32)
    return out


def count_params(input_type: str = "RGB", selective: bool = False, n_cls: int | None = None) -> int:
    return int(sum(np.prod(s) for _, s, _, _ in param_specs(input_type, selective, n_cls)))
