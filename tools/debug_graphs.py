"""Debug helper: per-step gradient norms and range words with / without HIP-graph replay."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402
from tests.test_gpu_model import build, train_step  # noqa: E402


def run(graphs, steps=5):
    os.environ["SELUNET_GRAPHS"] = "1" if graphs else "0"
    x, lab = make_batch(4, 64, seed=3)
    xt, lt = torch.tensor(x, device="cuda"), torch.tensor(lab, device="cuda")
    net = build(True, dtype=torch.float32)
    opt = S.Adam(net.parameters(), lr=1e-3)
    out = []
    for s in range(steps):
        h = train_step(net, opt, xt, lt, True, 2)
        eng = net._engine()
        words = None
        for lst in eng._plans.values():
            for e in lst:
                if e.ctx is not None and e.ctx.words:
                    words = {k: float(v.item()) for k, v in e.ctx.words.items()}
        out.append((h, words))
    return out


g = run(True)
e = run(False)
for s in range(5):
    hg, wg = g[s]
    he, we = e[s]
    diff = [k for k in hg["grads"] if not np.array_equal(hg["grads"][k], he["grads"][k])]
    print("step", s, "loss", hg["loss"], he["loss"], "ndiff", len(diff), diff[:4])
    for k in diff[:3]:
        print("   ", k, np.abs(hg["grads"][k]).max(), np.abs(he["grads"][k]).max())
    if wg and we:
        wd = {k: (wg[k], we[k]) for k in wg if wg[k] != we[k]}
        print("   words differing:", wd)
