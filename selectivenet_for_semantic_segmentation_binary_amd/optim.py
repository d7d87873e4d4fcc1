"""`torch.optim.Adam` drop-in (train.py:89-90, 207-209) with a single multi-tensor HIP kernel.

Same constructor, param_groups and state layout as torch.optim.Adam (state[p] = {'step',
'exp_avg', 'exp_avg_sq'}), so `optim.state_dict()` inside the reference checkpoint
({'net': ..., 'optim': ...}, utils/net_utils.py:5-9) loads into either class. Update rule
(torch's single-tensor algorithm, non-capturable):

    m = lerp(m, g, 1 - beta1);  v = beta2 v + (1 - beta2) g^2
    p -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)

with g += weight_decay * p first (L2, as torch.optim.Adam). One launch per param group: a
device table of {param, grad, exp_avg, exp_avg_sq, numel, chunk_begin} drives a grid of
4096-element chunks.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as K


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("amsgrad/maximize/capturable/differentiable are not used by train.py:90")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused)
        super().__init__(params, defaults)
        self._tables = {}

    def _table(self, gid, entries, device):
        key = (gid, tuple((e[0], e[1], e[2], e[3], e[4]) for e in entries))
        hit = self._tables.get(gid)
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        arr = (K.AdamTensor * len(entries))()
        chunk = 0
        for i, (p, g, m, v, n) in enumerate(entries):
            arr[i] = K.AdamTensor(p, g, m, v, n, chunk)
            chunk += -(-n // K.ADAM_CHUNK)
        host = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))),
                                dtype=torch.uint8)
        dev = host.to(device)
        self._tables[gid] = (key, dev, chunk)
        return dev, chunk

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gid, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                if p.device.type != "cuda" or p.dtype != torch.float32:
                    raise RuntimeError("the MI355X Adam updates fp32 cuda parameters only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if g is not p.grad:
                    p.grad = g
                by_step.setdefault(int(st["step"].item()), []).append(
                    (p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel(),
                     p.device))
            for step, entries in by_step.items():
                device = entries[0][5]
                table, chunks = self._table((gid, step if len(by_step) > 1 else -1),
                                            [e[:5] for e in entries], device)
                K.call("selunet_adam_step", K.ptr(table), len(entries), chunks, float(group["lr"]), float(beta1),
                       float(beta2), float(group["eps"]), float(group["weight_decay"]), step,
                       K.stream_ptr(device))
        return loss
