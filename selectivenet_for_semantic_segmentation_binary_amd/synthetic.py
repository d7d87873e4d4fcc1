"""Seeded synthetic tumor/benign H&E-like patches.

The reference trains on private WSI patches read by `PatchDataset`
(`utils/data_utils.py:170-236`). There is no data here, so benchmarks and parity
tests use a deterministic generator with the same shapes and the same
preprocessing as the reference:

* image uint8 RGB -> ``x / 255`` (`utils/data_utils.py:101-102`), then
  ``(x - 0.5) / 0.5`` (`Normalization`, `utils/data_utils.py:94-106`), then HWC->CHW
  (`ToTensor`, `utils/data_utils.py:160-168`), float32.
* label uint8 {0,255} -> ``(label / 255.0).astype(uint8)`` — truncation, so only 255
  maps to 1 (`utils/data_utils.py:220-221`) — then float32 for BCE (`train.py:189-191`).

Benign background is pinkish (≈(230,180,210)), tumor regions are 1–4 purple
(≈(150,90,160)) ellipses; per-pixel Gaussian noise σ≈20. ≈39% of patches are
"tumorable" (>10% tumor pixels), mirroring the reference's fold statistics
(`jupyters/tumor_label-based_data_split.ipynb`).
"""
from __future__ import annotations

import numpy as np

BENIGN_RGB = np.array([230.0, 180.0, 210.0])
TUMOR_RGB = np.array([150.0, 90.0, 160.0])


def make_patches(n: int, size: int = 256, seed: int = 0, tumorable_frac: float = 0.39):
    """Return (images uint8 [n,size,size,3], labels uint8 [n,size,size] in {0,255})."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    imgs = np.empty((n, size, size, 3), np.uint8)
    labs = np.zeros((n, size, size), np.uint8)
    for i in range(n):
        mask = np.zeros((size, size), bool)
        if rng.random() < tumorable_frac:
            k = int(rng.integers(1, 5))
            big = True
        else:
            k = int(rng.integers(0, 2))
            big = False
        for _ in range(k):
            cy, cx = rng.uniform(0, size, 2)
            scale = size * (rng.uniform(0.15, 0.35) if big else rng.uniform(0.03, 0.08))
            ay, ax = scale * rng.uniform(0.6, 1.4, 2)
            th = rng.uniform(0, np.pi)
            c, s = np.cos(th), np.sin(th)
            dy, dx = yy - cy, xx - cx
            u = (c * dx + s * dy) / ax
            v = (-s * dx + c * dy) / ay
            mask |= (u * u + v * v) <= 1.0
        base = np.where(mask[..., None], TUMOR_RGB, BENIGN_RGB)
        noise = rng.normal(0.0, 20.0, size=(size, size, 3))
        imgs[i] = np.clip(base + noise, 0, 255).astype(np.uint8)
        labs[i] = np.where(mask, 255, 0).astype(np.uint8)
    return imgs, labs


def make_patches_hard(n: int, size: int = 256, seed: int = 0, contrast: float = 0.35, noise: float = 28.0,
                      texture: float = 20.0, decoys: int = 6, tumorable_frac: float = 0.39):
    """A harder task for the mIoU parity run (tests/test_gpu_train.py): the tumor colour lies only
    `contrast` of the way from the benign colour to the purple of make_patches, under per-pixel noise
    `noise` and a smooth per-channel stain texture of amplitude `texture` shared by both classes, and
    every patch carries up to `decoys` small unlabelled blobs in the tumor colour (benign nuclei), so
    a per-pixel colour rule fails and the network must use shape and context. Labels as make_patches:
    1-4 large ellipses in 'tumorable' patches, 0-1 small ones otherwise."""
    from scipy.ndimage import zoom

    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    tumor = BENIGN_RGB + contrast * (TUMOR_RGB - BENIGN_RGB)
    imgs = np.empty((n, size, size, 3), np.uint8)
    labs = np.zeros((n, size, size), np.uint8)

    def ellipse(scale):
        cy, cx = rng.uniform(0, size, 2)
        ay, ax = scale * rng.uniform(0.6, 1.4, 2)
        th = rng.uniform(0, np.pi)
        c, s = np.cos(th), np.sin(th)
        dy, dx = yy - cy, xx - cx
        u = (c * dx + s * dy) / ax
        v = (-s * dx + c * dy) / ay
        return (u * u + v * v) <= 1.0

    g = max(2, size // 32)
    for i in range(n):
        mask = np.zeros((size, size), bool)
        big = rng.random() < tumorable_frac
        for _ in range(int(rng.integers(1, 5)) if big else int(rng.integers(0, 2))):
            mask |= ellipse(size * (rng.uniform(0.15, 0.35) if big else rng.uniform(0.03, 0.08)))
        decoy = np.zeros((size, size), bool)
        for _ in range(int(rng.integers(0, decoys + 1))):
            decoy |= ellipse(size * rng.uniform(0.02, 0.05))
        base = np.where((mask | decoy)[..., None], tumor, BENIGN_RGB)
        tex = zoom(rng.normal(0.0, texture, size=(g, g, 3)), (size / g, size / g, 1), order=1)[:size, :size]
        img = base + tex + rng.normal(0.0, noise, size=(size, size, 3))
        imgs[i] = np.clip(img, 0, 255).astype(np.uint8)
        labs[i] = np.where(mask, 255, 0).astype(np.uint8)
    return imgs, labs


def preprocess(imgs: np.ndarray, labs: np.ndarray):
    """Reference preprocessing -> (x float32 [N,3,H,W], label float32 [N,H,W])."""
    x = imgs.astype(np.float64) / 255.0
    x = x.astype(np.float32)
    x = (x - 0.5) / 0.5
    x = np.ascontiguousarray(x.transpose(0, 3, 1, 2)).astype(np.float32)
    lab = (labs / 255.0).astype(np.uint8).astype(np.float32)
    return x, lab


def make_batch(n: int, size: int = 256, seed: int = 0):
    imgs, labs = make_patches(n, size, seed)
    return preprocess(imgs, labs)
