"""ORACLE — CPU restatement of the reference's patch data path.

TEST INFRASTRUCTURE ONLY. Imported solely by `tests/` as the checker of the package's data path
(`data.decode_patch_list`, `data.construct_train_valid/construct_test`, `data.BatchLoader` +
`selunet_prep_batch`); the product path never imports it.

What it restates, op by op in numpy/PIL (written from the reference's semantics, not copied):

* `PatchDataset.__getitem__` (`utils/data_utils.py:203-236`): PIL open of
  `{data_dir}/{patch_mag}x_{patch_size}/{input}` (no mode conversion) and of the label with
  `.convert("L")`; `input / 255.0` and `label / 255.0` in float64, then `input.astype(float32)`,
  `label.astype(uint8)` (truncation: only 255 becomes 1), the id `input.split('_input')[0]`.
* `Normalization(mean=0.5, std=0.5)` (`utils/data_utils.py:94-106`): `(input - 0.5) / 0.5` on the
  float32 array (numpy keeps float32 for a Python-float operand).
* `RandomFlip` (`utils/data_utils.py:108-125`): `np.fliplr` when the first draw > 0.5, then
  `np.flipud` when the second draw > 0.5, on input and label alike. The draws are passed in
  (`flips` bit 0 = lr, bit 1 = ud), since the loader's random stream is its own.
* `ToTensor` (`utils/data_utils.py:160-168`): HWC -> CHW float32; label int64, turned into float32
  for the BCE losses by the loop (`train.py:187-191`).
* `split_train_valid` / `construct_train_valid` / `construct_test` (`utils/data_utils.py:49-86`)
  with the module-level `np.random.seed(42)` they draw from (`utils/data_utils.py:50`): the global
  numpy stream is seeded here exactly as importing the reference module does.

Parity pinning: the reference's data module is not importable in this image (it imports `cv2`,
`skimage` and `torchvision`, all absent — SURVEY.md §8c), and the reference ships no data
fixtures, so this restatement is **parity unpinned** by reference outputs; it is pinned to the
reference's source semantics above (every call is the same numpy/PIL call the reference makes) and
checked by `tests/test_data_oracle.py` against hand-computed values.
"""
from __future__ import annotations

import os

import numpy as np


def read_patch(data_dir, input_file, label_file, patch_mag=200, patch_size=256):
    """utils/data_utils.py:213-221 -> (input float32 [H,W,3] in [0,1], label uint8 [H,W], id)."""
    from PIL import Image

    assert input_file.split("_input")[0] == label_file.split("_label")[0]
    root = os.path.join(data_dir, f"{patch_mag}x_{patch_size}")
    inp = np.array(Image.open(os.path.join(root, input_file)))
    lab = np.array(Image.open(os.path.join(root, label_file)).convert("L"))
    inp, lab = inp / 255.0, lab / 255.0
    return inp.astype(np.float32), lab.astype(np.uint8), input_file.split("_input")[0]


HED_FROM_RGB_H = (1.8779827368521353, -0.06590806222356332, -0.6019073634392891)  # inv(rgb_from_hed)[:, 0]


def rgb2gh(rgb):
    """RGB2GH (utils/data_utils.py:13-27) restated without cv2/skimage: cv2.cvtColor(RGB2GRAY) of a
    float32 image = 0.299 R + 0.587 G + 0.114 B; skimage.color.separate_stains(rgb, hed_from_rgb)
    (skimage >= 0.19 form) = (log(max(rgb, 1e-6)) / log(1e-6)) @ hed_from_rgb, clamped at 0, column
    0; min-max normalised with the reference's constants. Parity unpinned (neither library is
    importable here, and the skimage form is version-dependent)."""
    r, g, b = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    gray = r * np.float32(0.299) + g * np.float32(0.587) + b * np.float32(0.114)
    q = np.log(np.maximum(rgb, np.float32(1e-6))) / np.float32(np.log(np.float32(1e-6)))
    st = np.maximum(q.astype(np.float64) @ np.array(HED_FROM_RGB_H), 0.0)
    h = (st - (-0.66781543)) / (1.87798274 - (-0.66781543))
    return np.concatenate((gray[..., None], h[..., None]), axis=-1).astype(np.float32)


def h_rgb(rgb):
    """H_RGB (utils/data_utils.py:29-41) restated: the hematoxylin stain of separate_stains (as in
    rgb2gh), recombined alone by skimage.color.combine_stains (>= 0.19 form): rgb =
    clip(exp(-(stains * -log(1e-6)) @ rgb_from_hed), 0, 1) with stains = (h, 0, 0). Parity unpinned."""
    q = np.log(np.maximum(rgb, np.float32(1e-6))) / np.float32(np.log(np.float32(1e-6)))
    h = np.maximum(q.astype(np.float64) @ np.array(HED_FROM_RGB_H), 0.0)
    out = np.exp(-(h[..., None] * -np.log(1e-6)) * np.array([0.65, 0.70, 0.29]))
    return np.clip(out, 0, 1).astype(np.float32)


def transform(inp, lab, flips=0, train=True):
    """Normalization -> [RandomFlip] -> ToTensor (train.py:355-356) -> (x float32 [3,H,W],
    label float32 [H,W] as train.py:189-191 hands it to BCEWithLogitsLoss)."""
    inp = (inp - 0.5) / 0.5
    if train:
        if flips & 1:
            lab = np.fliplr(lab).copy()
            inp = np.fliplr(inp)
        if flips & 2:
            lab = np.flipud(lab).copy()
            inp = np.flipud(inp)
    x = inp.transpose((2, 0, 1)).astype(np.float32)
    return x, lab.astype(np.int64).astype(np.float32)


def split_train_valid(lst, valid_ratio=0.2):
    """utils/data_utils.py:52-56 (draws from the global numpy stream)."""
    total_n = len(lst)
    valid_idx = np.random.choice(total_n, size=int(total_n * valid_ratio), replace=False)
    train_idx = np.setdiff1d([i for i in range(total_n)], valid_idx)
    return lst[train_idx], lst[valid_idx]


def construct_train_valid(data_dir, test_fold=5):
    """utils/data_utils.py:58-76, after the module import's np.random.seed(42) (:50)."""
    np.random.seed(42)
    folds = [1, 2, 3, 4, 5]
    folds.remove(test_fold)
    tum = np.concatenate([np.load(f"{data_dir}/{i}-fold_tumorable_data.npy") for i in folds])
    non = np.concatenate([np.load(f"{data_dir}/{i}-fold_non_tumorable_data.npy") for i in folds])
    t_train, t_valid = split_train_valid(tum, 0.2)
    n_train, n_valid = split_train_valid(non, 0.2)
    return np.vstack([t_train, n_train]), np.vstack([t_valid, n_valid])


def construct_test(data_dir, test_fold=1):
    """utils/data_utils.py:78-86."""
    tum = np.array(np.load(f"{data_dir}/{test_fold}-fold_tumorable_data.npy"))
    non = np.array(np.load(f"{data_dir}/{test_fold}-fold_non_tumorable_data.npy"))
    return np.vstack([tum, non])


def batch(data_dir, pairs, flips=None, train=True, patch_mag=200, patch_size=256, input_type="RGB"):
    """DataLoader's default collate of __getitem__ + transform over `pairs` (train.py:378-381)
    -> (x float32 [N,3,H,W], label float32 [N,H,W], ids)."""
    xs, ls, ids = [], [], []
    for i, (a, b) in enumerate(pairs):
        inp, lab, pid = read_patch(data_dir, str(a), str(b), patch_mag, patch_size)
        if input_type == "GH":
            inp = rgb2gh(inp)
        elif input_type == "H_RGB":
            inp = h_rgb(inp)
        x, t = transform(inp, lab, 0 if flips is None else int(flips[i]), train)
        xs.append(x)
        ls.append(t)
        ids.append(pid)
    return np.stack(xs), np.stack(ls), ids
