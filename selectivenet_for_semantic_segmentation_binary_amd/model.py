"""Drop-in `UNet_B` / `CBR_2D` (reference: model.py:9-103) backed by the MI355X kernels.

Same constructor signature (`UNet_B(input_type='RGB', selective=False)`), same submodule
names, parameter shapes and registration order (so `state_dict()` keys, checkpoints and Adam
state indices are interchangeable with the reference), same forward contract: `[N,C,H,W]`
fp32 in, `(N,H,W)` logits out, or the `(out, select, aux)` triple when selective
(model.py:98-103). The modules inside `CBR_2D` are parameter containers only; the forward
runs entirely in libselunet.so through one autograd.Function (`_UNetBFunction`).

Extra keyword (not in the reference): `compute_dtype` — torch.float32 (default, the parity
configuration: fp32 tensors; in training the 3x3 convolutions run on split-fp16 operands with an
error at or below the exact fp32 MFMA's, SELUNET_X2=0 selects exact fp32 MFMA products) or
torch.bfloat16 (bf16 operands, fp32 accumulation, statistics, losses and master weights).
"""
from __future__ import annotations

import math
import weakref

import torch
import torch.nn as nn

from . import _lib as K
from . import layout as LY
from . import parallel
from .engine import Engine


class _Conv2dParams(nn.Module):
    """Holds Conv2d(in, out, k) parameters exactly as nn.Conv2d registers them."""

    def __init__(self, in_ch, out_ch, k):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = in_ch, out_ch, (k, k)
        self.weight = nn.Parameter(torch.empty(out_ch, in_ch, k, k))
        self.bias = nn.Parameter(torch.empty(out_ch))
        self.reset_parameters()

    def reset_parameters(self):
        # torch.nn.Conv2d default init (kaiming_uniform_(a=sqrt(5)) and fan_in-bounded bias)
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(self.weight[0].numel())
        nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):  # pragma: no cover - the whole network runs as one fused Function
        raise RuntimeError("submodules of the MI355X UNet_B are parameter containers; call the UNet_B module")


class _ConvTranspose2dParams(_Conv2dParams):
    def __init__(self, in_ch, out_ch, k):
        nn.Module.__init__(self)
        self.in_channels, self.out_channels, self.kernel_size = in_ch, out_ch, (k, k)
        self.weight = nn.Parameter(torch.empty(in_ch, out_ch, k, k))
        self.bias = nn.Parameter(torch.empty(out_ch))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(out_ch * k * k)
        nn.init.uniform_(self.bias, -bound, bound)


class _BatchNorm2dParams(nn.Module):
    """BatchNorm2d(num_features) parameters and buffers (eps 1e-5, momentum 0.1)."""

    def __init__(self, c):
        super().__init__()
        self.num_features, self.eps, self.momentum = c, 1e-5, 0.1
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def forward(self, x):  # pragma: no cover
        raise RuntimeError("parameter container")


class _ReLU(nn.Module):
    def forward(self, x):  # pragma: no cover
        raise RuntimeError("parameter container")


def CBR_2D(in_ch, out_ch, k_size=3, stride=1, padding=1, bias=True):
    """model.py:9-15: Sequential(Conv2d, BatchNorm2d, ReLU) — here as parameter containers
    (only the reference's arguments k_size=3, stride=1, padding=1, bias=True are supported)."""
    if (k_size, stride, padding, bias) != (3, 1, 1, True):
        raise NotImplementedError("the MI355X CBR_2D implements conv3x3 / stride 1 / pad 1 / bias (model.py:9)")
    return nn.Sequential(_Conv2dParams(in_ch, out_ch, 3), _BatchNorm2dParams(out_ch), _ReLU())


class _UNetBFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        names = module._param_names
        P = dict(zip(names, params))
        B = dict(module.named_buffers())
        training = module.training
        if not training and parallel.is_initialized():
            parallel.broadcast_buffers(module)  # DataParallel replicas read device 0's buffers
        eng = module._engine()
        need_bwd = training and any(ctx.needs_input_grad[2:])
        outs, ectx = eng.forward(x.contiguous(), P, B, module.selective, training, need_backward=need_bwd,
                                 ce_heads=module._ce_heads)
        if need_bwd:
            ctx.ectx = ectx
            ctx.eng = eng
            ctx.names = names
            ctx.P = P
            # a graph freed without backward must hand the engine's launch plan back
            ctx.release = weakref.finalize(ctx, Engine.release, ectx)
        else:
            ctx.ectx = None
        return outs if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, *g_heads):
        if ctx.ectx is None:
            raise RuntimeError("UNet_B backward needs a training-mode forward with grad enabled")
        names, P = ctx.names, ctx.P
        dev = g_heads[0].device if g_heads[0] is not None else next(iter(P.values())).device
        total = sum(P[n].numel() for n in names)
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        G, off, layout = {}, 0, []
        for n in names:
            k = P[n].numel()
            G[n] = flat[off:off + k].view(P[n].shape)
            layout.append((n, off, k))
            off += k
        # DataParallel reduce-add of the replica gradients: bucketed all-reduces issued while the
        # backward of the shallower layers still runs
        emu = parallel.overlap_emulation()
        bucketer = (parallel.GradBucketer(flat, layout, parallel.bucket_elems(), emulate=emu) if parallel.is_initialized() or emu is not None
                    else None)
        ctx.eng.backward(ctx.ectx, P, G, list(g_heads), flat, on_grads=bucketer.ready if bucketer else None)
        ctx.release.detach()
        ctx.ectx = None
        if bucketer is not None:
            bucketer.finish()
        return (None, None, *[G[n] for n in names])


class _UNetBase(nn.Module):
    """The encoder-decoder shared by UNet_B (model.py:18-103) and the CE UNet (model.py:105-191);
    they differ only in the 1x1 heads (n_cls None: 1-channel heads)."""

    def __init__(self, input_type="RGB", selective=False, compute_dtype=torch.float32, n_cls=None):
        super().__init__()
        self.selective = selective
        input_ch = LY.input_channels(input_type)
        self.compute_dtype = compute_dtype

        self.encoder_layer_1_1 = CBR_2D(in_ch=input_ch, out_ch=64)
        self.encoder_layer_1_2 = CBR_2D(in_ch=64, out_ch=64)
        self.pool1 = nn.Identity()
        self.encoder_layer_2_1 = CBR_2D(in_ch=64, out_ch=128)
        self.encoder_layer_2_2 = CBR_2D(in_ch=128, out_ch=128)
        self.pool2 = nn.Identity()
        self.encoder_layer_3_1 = CBR_2D(in_ch=128, out_ch=256)
        self.encoder_layer_3_2 = CBR_2D(in_ch=256, out_ch=256)
        self.pool3 = nn.Identity()
        self.decoder_layer_4_2 = CBR_2D(in_ch=256, out_ch=512)
        self.decoder_layer_4_1 = CBR_2D(in_ch=512, out_ch=512)
        self.unpool3 = _ConvTranspose2dParams(512, 256, 2)
        self.decoder_layer_3_2 = CBR_2D(in_ch=512, out_ch=256)
        self.decoder_layer_3_1 = CBR_2D(in_ch=256, out_ch=256)
        self.unpool2 = _ConvTranspose2dParams(256, 128, 2)
        self.decoder_layer_2_2 = CBR_2D(in_ch=256, out_ch=128)
        self.decoder_layer_2_1 = CBR_2D(in_ch=128, out_ch=128)
        self.unpool1 = _ConvTranspose2dParams(128, 64, 2)
        self.decoder_layer_1_2 = CBR_2D(in_ch=128, out_ch=64)
        self.decoder_layer_1_1 = CBR_2D(in_ch=64, out_ch=64)
        for h, c in LY.head_channels(selective, n_cls):
            setattr(self, h, _Conv2dParams(64, c, 1))
        self._ce_heads = None if n_cls is None else LY.head_channels(selective, n_cls)
        self._param_names = [n for n, _ in self.named_parameters()]
        self._engines = {}

    def _engine(self):
        e = self._engines.get(self.compute_dtype)
        if e is None:
            e = self._engines[self.compute_dtype] = Engine(self.compute_dtype)
        return e

    def forward(self, x):
        if x.device.type != "cuda":
            raise RuntimeError("the MI355X UNet_B runs on the GPU only (no CPU fallback); move the model and "
                               "input to a cuda device")
        K.load()
        params = [p for _, p in self.named_parameters()]
        if x.dtype != torch.float32:
            x = x.float()
        return _UNetBFunction.apply(x, self, *params)


class UNet_B(_UNetBase):
    """model.py:18-103 UNet for BCE loss, optionally SelectiveNet (selection + aux heads):
    [N, C_in, H, W] -> (N, H, W) logits, or (out, select, aux) each (N, H, W)."""

    def __init__(self, input_type="RGB", selective=False, compute_dtype=torch.float32):
        super().__init__(input_type, selective, compute_dtype)


class UNet(_UNetBase):
    """model.py:105-191 UNet for CE loss: conv1x1 64 -> n_cls; when selective conv_select 64 -> 2 and
    conv_aux 64 -> n_cls. [N, C_in, H, W] -> (N, n_cls, H, W) logits, or (out, select, aux) with
    select (N, 2, H, W) (model.py:182-189). n_cls + 2 + n_cls <= 8 output channels (n_cls <= 3
    selective, <= 8 otherwise) — the reference trains with n_cls = 2 (train.py:23)."""

    def __init__(self, input_type="RGB", n_cls=2, selective=False, compute_dtype=torch.float32):
        if n_cls < 1 or sum(c for _, c in LY.head_channels(selective, n_cls)) > 8:
            raise ValueError(f"n_cls={n_cls}: the heads may have at most 8 output channels in total")
        super().__init__(input_type, selective, compute_dtype, n_cls=n_cls)
        self.n_cls = n_cls
