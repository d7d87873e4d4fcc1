"""mIoU run of the reference training loop on other fp32 realisations (test infrastructure, GPU).

VERDICT r5 item 1: is the HIP fp32 path's validation mIoU on miou_sel_256h.npz (0.9265 against the
reference run's 0.9284) a bias of our kernels or one draw of a chaotic 16-epoch run? This script trains
the same loop as tests/golden/make_golden.py::miou_fixture (train.py:183-241: BCEWithLogits aux +
calc_selective_risk_image_b with s_lamb 2, torch Adam lr 1e-3, CosineAnnealingLR to 1e-5 stepped per
epoch, train.py:100-101,246-250; eval-mode mIoU, utils/compute_metric.py:60-65) through:

* ``--impl torch``: the oracle's restatement of UNet_B (oracle/unet_b_cpu.py, pinned against the
  reference) on torch's own GPU kernels (MIOpen convolutions) in fp32 or fp64 — a third fp32
  implementation beside the reference's CPU run and ours, and an fp64 trajectory; with ``--conv-noise
  k1,k2,..`` each member multiplies every convolution output (3x3, transposed, 1x1 heads: the
  reference's Conv2d / ConvTranspose2d modules) by (1 + 3e-7 N(0,1)) in every training forward, as
  make_golden.py miou256c_member does on the CPU reference;
* ``--impl hip``: the package's HIP path (whichever fp32 kernels the environment selects:
  SELUNET_X2=0 is the exact-fp32 MFMA path), optionally with the same input perturbation as the
  reference's members.

Writes one JSON line per run to stdout and appends it to --out. The runs are data for the mIoU gate
(tests/test_gpu_train.py); nothing here is product code.

    python tests/golden/miou_gpu_ensemble.py --fixture miou_sel_256h.npz --impl torch --dtype f32 \
        --conv-noise 0,1,2,3 --out gpurun_out/miou_torch.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from selectivenet_for_semantic_segmentation_binary_amd.metrics import SegMetrics, mean_iou  # noqa: E402
from tests import _golden as G  # noqa: E402
from tests.test_gpu_train import _miou_data  # noqa: E402

DEV = "cuda"


class _NoisyConvF:
    """torch.nn.functional with conv2d / conv_transpose2d outputs perturbed by (1 + eps N(0,1))."""

    def __init__(self, eps, seed):
        self.eps = eps
        self.gen = torch.Generator(device=DEV).manual_seed(5000 + seed)

    def _noisy(self, out):
        z = torch.randn(out.shape, generator=self.gen, device=out.device, dtype=torch.float64).to(out.dtype)
        return out + out * (self.eps * z)

    def conv2d(self, *a, **k):
        return self._noisy(F.conv2d(*a, **k))

    def conv_transpose2d(self, *a, **k):
        return self._noisy(F.conv_transpose2d(*a, **k))

    def __getattr__(self, name):
        return getattr(F, name)


def run_torch(d, data, dtype, noise, eps):
    from oracle import unet_b_cpu as O
    (xtr, ltr), (xva, lva) = data
    bs, epochs, lamb = int(d["meta_bs"]), int(d["meta_epochs"]), int(d["meta_lamb"])
    cmin = float(d["meta_cosine_min"]) if "meta_cosine_min" in d.files else 0.0
    params, buffers = O.make_state(int(d["meta_seed"]), "RGB", True)
    params = {k: v.detach().to(DEV, dtype).requires_grad_(True) for k, v in params.items()}
    buffers = {k: (v.to(DEV, dtype) if v.is_floating_point() else v.to(DEV)) for k, v in buffers.items()}
    opt = torch.optim.Adam(list(params.values()), lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=epochs, eta_min=cmin) if cmin > 0 else None
    xt, lt = torch.tensor(xtr, device=DEV, dtype=dtype), torch.tensor(ltr, device=DEV, dtype=dtype)
    tr = SegMetrics(DEV, selective=True, rule="train")
    f_saved = O.F
    if noise:
        O.F = _NoisyConvF(eps, noise)
    try:
        for ep in range(epochs):
            if ep > 0 and sched is not None:
                sched.step()
            for b0 in range(0, xt.shape[0], bs):
                x, lab = xt[b0:b0 + bs], lt[b0:b0 + bs]
                o, s, a = O.forward(params, buffers, x, True, training=True)
                loss = O.bce_with_logits_mean(a, lab) + O.selective_risk_b_stable(o, s, lab, lamb=lamb)[0]
                opt.zero_grad()
                loss.backward()
                opt.step()
                tr.add_batch(o.detach().float(), lab.float(), s.detach().float())
    finally:
        O.F = f_saved
    vs, vp = SegMetrics(DEV, selective=True, rule="train"), SegMetrics(DEV, selective=False, rule="train")
    xv, lv = torch.tensor(xva, device=DEV, dtype=dtype), torch.tensor(lva, device=DEV)
    with torch.no_grad():
        for b0 in range(0, xv.shape[0], bs):
            o, s, _ = O.forward(params, buffers, xv[b0:b0 + bs], True, training=False)
            vs.add_batch(o.float(), lv[b0:b0 + bs], s.float())
            vp.add_batch(o.float(), lv[b0:b0 + bs], s.float())
    return tr, vs, vp, float(loss.item())


def run_hip(d, data, member):
    from tests.test_gpu_train import miou_run
    return miou_run(d, data, torch.float32, member)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="miou_sel_256h.npz")
    ap.add_argument("--impl", choices=("torch", "hip"), default="torch")
    ap.add_argument("--dtype", choices=("f32", "f64"), default="f32")
    ap.add_argument("--conv-noise", default="0", help="comma list of conv-noise members (0: none) [torch]")
    ap.add_argument("--members", default="0", help="comma list of input-perturbed members (0: none) [hip]")
    ap.add_argument("--eps", type=float, default=3e-7)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    d = G.load(a.fixture)
    data = _miou_data(d)
    tag = a.impl if a.impl == "torch" else ("hip-exact" if os.environ.get("SELUNET_X2") == "0" else "hip-split")
    ks = [int(v) for v in (a.conv_noise if a.impl == "torch" else a.members).split(",")]
    for k in ks:
        t0 = time.time()
        if a.impl == "torch":
            tr, vs, vp, last = run_torch(d, data, torch.float64 if a.dtype == "f64" else torch.float32, k, a.eps)
            sel, total = vs.selected_total()
            rec = {"fixture": a.fixture, "impl": tag, "dtype": a.dtype, "conv_noise": k, "eps": a.eps,
                   "train_miou": mean_iou(tr.confusion_matrix()), "val_miou": mean_iou(vp.confusion_matrix()),
                   "val_miou_selective": mean_iou(vs.confusion_matrix()), "val_selected": int(sel),
                   "val_total": int(total), "last_loss": last}
        else:
            rec = {"fixture": a.fixture, "impl": tag, "dtype": "f32", **run_hip(d, data, k)}
        rec.update(ref_val_miou=float(d["val_miou"]), ref_val_miou_selective=float(d["val_miou_selective"]),
                   seconds=round(time.time() - t0, 1))
        line = json.dumps(rec)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
