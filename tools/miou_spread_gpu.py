"""How chaotic is the validation mIoU of a short training run? (profiling / study tool, GPU)

Trains the HIP SelectiveUNet_B (fp32, split-fp16 convolutions) with the reference's loop
(train.py:183-241: BCEWithLogits aux + calc_selective_risk_image_b, Adam) on seeded synthetic
patches, K times with the training inputs perturbed by 1e-7 relative (member 0 unperturbed), and
prints each member's training-phase and eval-mode validation mIoU and the spread — the quantity
tests/golden/make_golden.py::miou_spread measures on the reference, found here in seconds per run.

    python tools/miou_spread_gpu.py --n-train 128 --n-val 256 --size 256 --bs 16 --epochs 4 --lr 1e-3 -k 8
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.metrics import SegMetrics, mean_iou  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_patches, make_patches_hard, preprocess  # noqa: E402


def run(xtr, ltr, xva, lva, a, member):
    if member:
        rng = np.random.Generator(np.random.PCG64(1000 + member))
        xtr = (xtr.astype(np.float64) * (1.0 + 1e-7 * rng.standard_normal(xtr.shape))).astype(np.float32)
    dev = "cuda"
    net = S.UNet_B("RGB", selective=True)
    p = L.seeded_params(0, "RGB", True)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(dev).train()
    opt = S.Adam(net.parameters(), lr=a.lr)
    loss_a = S.BCEWithLogitsLoss()
    xt, lt = torch.tensor(xtr, device=dev), torch.tensor(ltr, device=dev)
    tr = SegMetrics(dev, selective=True, rule="train")
    for ep in range(a.epochs):
        if a.lr_decay and ep == a.epochs // 2:
            for g in opt.param_groups:
                g["lr"] = a.lr * a.lr_decay
        if a.cosine:  # train.py:100-101,246-250: CosineAnnealingLR(T_max=epochs, eta_min=lr_min), per epoch
            lr = a.lr_min + (a.lr - a.lr_min) * (1 + np.cos(np.pi * ep / a.epochs)) / 2
            for g in opt.param_groups:
                g["lr"] = lr
        for b0 in range(0, xt.shape[0], a.bs):
            x, lab = xt[b0:b0 + a.bs], lt[b0:b0 + a.bs]
            o, s, ax = net(x)
            loss = loss_a(ax, lab) + S.calc_selective_risk_image_b(o, s, target=lab, lamb=a.lamb)[0]
            opt.zero_grad()
            loss.backward()
            opt.step()
            tr.add_batch(o.detach(), lab, s.detach())
    net.eval()
    vp = SegMetrics(dev, selective=False, rule="train")
    vs = SegMetrics(dev, selective=True, rule="train")
    xv, lv = torch.tensor(xva, device=dev), torch.tensor(lva, device=dev)
    with torch.no_grad():
        for b0 in range(0, xv.shape[0], a.bs):
            o, s, _ = net(xv[b0:b0 + a.bs])
            vp.add_batch(o, lv[b0:b0 + a.bs], s)
            vs.add_batch(o, lv[b0:b0 + a.bs], s)
    cms = vs.confusion_matrix()
    return (mean_iou(tr.confusion_matrix()), mean_iou(vp.confusion_matrix()), float(loss.item()), mean_iou(cms),
            float(np.asarray(cms).sum()) / lva.size, float(np.asarray(cms)[1].sum()) / max(1.0, float(lva.sum())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-train", type=int, default=128)
    ap.add_argument("--n-val", type=int, default=256)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--lr-decay", type=float, default=0.0, help="multiply lr by this at half the epochs")
    ap.add_argument("--lamb", type=float, default=2)
    ap.add_argument("--cosine", action="store_true", help="cosine-annealed lr per epoch down to --lr-min")
    ap.add_argument("--lr-min", type=float, default=1e-5)
    ap.add_argument("-k", type=int, default=8)
    ap.add_argument("--hard", default="", help="';'-separated make_patches_hard settings "
                    "'contrast,noise,texture,decoys[,tumorable_frac]' to sweep (empty: make_patches)")
    a = ap.parse_args()
    for cfg in (a.hard.split(";") if a.hard else [None]):
        if cfg:
            vals = [float(v) for v in cfg.split(",")]
            c, nz, tx, dc = vals[:4]
            tf = vals[4] if len(vals) > 4 else 0.39
            gen = lambda n, seed: make_patches_hard(n, a.size, seed=seed, contrast=c, noise=nz, texture=tx,  # noqa
                                                    decoys=int(dc), tumorable_frac=tf)
        else:
            gen = lambda n, seed: make_patches(n, a.size, seed=seed)  # noqa: E731
        xtr, ltr = preprocess(*gen(a.n_train, 2024))
        xva, lva = preprocess(*gen(a.n_val, 2025))
        res = [run(xtr, ltr, xva, lva, a, m) for m in range(a.k + 1)]
        tr = np.array([r[0] for r in res])
        va = np.array([r[1] for r in res])
        vs = np.array([r[3] for r in res])
        print(f"cfg {vars(a)} hard={cfg}")
        print("val selective mIoU", np.round(vs, 5), "coverage", [round(r[4], 4) for r in res],
              "tumour pixels kept", [round(r[5], 4) for r in res], "tumour fraction", round(float(lva.mean()), 4))
        print("train mIoU", np.round(tr, 5), "val mIoU", np.round(va, 5), "final loss", [round(r[2], 4) for r in res])
        print(f"SPREAD hard={cfg} train {np.abs(tr[1:] - tr[0]).max():.5f} val {np.abs(va[1:] - va[0]).max():.5f} "
              f"val range {va.max() - va.min():.5f} val0 {va[0]:.5f} | selective spread "
              f"{np.abs(vs[1:] - vs[0]).max() if len(vs) > 1 else 0:.5f} sel0 {vs[0]:.5f}", flush=True)


if __name__ == "__main__":
    main()
