"""A tiny on-disk patch dataset in the reference's layout (utils/data_utils.py:49-86, 170-221):
`{root}/{k}-fold_{tumorable,non_tumorable}_data.npy` lists of (input .jpg, label .png) names and the
files under `{root}/{mag}x_{size}/`, written with PIL from the seeded synthetic generator."""
import os

import numpy as np

from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_patches


def make_patch_dir(root, per_fold=6, size=32, mag=200, seed=0):
    from PIL import Image

    sub = os.path.join(root, f"{mag}x_{size}")
    os.makedirs(sub, exist_ok=True)
    imgs, labs = make_patches(5 * per_fold, size, seed)
    k = 0
    for fold in range(1, 6):
        tum, non = [], []
        for j in range(per_fold):
            a, b = f"slide{fold}_{j * 256}_{k}_input.jpg", f"slide{fold}_{j * 256}_{k}_label.png"
            Image.fromarray(imgs[k]).save(os.path.join(sub, a), quality=90)
            lab = labs[k].copy()
            lab[0, : size // 4] = 254  # non-255 mask values: truncated to 0 by label/255 -> uint8
            Image.fromarray(lab).save(os.path.join(sub, b))
            (tum if labs[k].mean() > 25 else non).append((a, b))
            k += 1
        for name, lst in (("tumorable", tum), ("non_tumorable", non)):
            np.save(os.path.join(root, f"{fold}-fold_{name}_data.npy"), np.array(lst, dtype="<U64").reshape(-1, 2))
    return root
