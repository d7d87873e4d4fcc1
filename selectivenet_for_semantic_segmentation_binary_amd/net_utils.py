"""Checkpoint helpers with the reference's file layout (utils/net_utils.py:5-53, train.py:385).

A checkpoint is `{'net': model.state_dict(), 'optim': optimizer.state_dict()}` saved as
`{ckpt_dir}/model_epoch{E}.pth`. Keys written by a DataParallel model carry a `module.` prefix,
which the loaders strip, so checkpoints move freely between the reference and this package in
both directions (the UNet_B state_dict keys and the Adam state layout are the reference's).
Only rank 0 should save under data parallelism (its BN buffers are DataParallel's replica 0).
Loading uses `torch.load(..., weights_only=True)`: a checkpoint is tensors and plain containers.
"""
from __future__ import annotations

import os
import re
from collections import OrderedDict

import torch


def net_save(ckpt_dir, net, optim, epoch):
    """utils/net_utils.py:5-9."""
    os.makedirs(ckpt_dir, exist_ok=True)
    torch.save({"net": net.state_dict(), "optim": optim.state_dict()}, os.path.join(ckpt_dir, f"model_epoch{epoch}.pth"))


def remove_module(ckpt):
    """utils/net_utils.py:11-16: strip DataParallel's `module.` prefix from ckpt['net']."""
    return OrderedDict((k.replace("module.", ""), v) for k, v in ckpt["net"].items())


def _epoch_key(fname):
    digits = "".join(ch for ch in fname if ch.isdigit())
    return int(digits) if digits else -1


def _load(path, device):
    return torch.load(path, map_location=device if device is not None else "cpu", weights_only=True)


def net_train_load(ckpt_dir, net, optim, device=None):
    """utils/net_utils.py:18-40: resume from the newest checkpoint (ordered by the digits in the
    file name, as the reference sorts); returns (net, optim, epoch), epoch 0 if none exists."""
    if not os.path.exists(ckpt_dir):
        return net, optim, 0
    names = sorted(os.listdir(ckpt_dir), key=_epoch_key)
    if not names:
        return net, optim, 0
    ckpt = _load(os.path.join(ckpt_dir, names[-1]), device)
    ckpt["net"] = remove_module(ckpt)
    net.load_state_dict(ckpt["net"])
    optim.load_state_dict(ckpt["optim"])
    m = re.search(r"epoch(\d+)\.pth", names[-1])
    epoch = int(m.group(1)) if m else _epoch_key(names[-1])
    return net, optim, epoch


def net_test_load(model_path, net, device=None):
    """utils/net_utils.py:42-53."""
    ckpt = _load(model_path, device)
    ckpt["net"] = remove_module(ckpt)
    net.load_state_dict(ckpt["net"])
    return net
