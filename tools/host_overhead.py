"""Host enqueue cost of one training step vs its GPU time at small per-GPU batches (the 8-GPU
strong-scaling regime: global 128 -> 16 images per GPU) — profiling tool.

    python tools/host_overhead.py [--batch 16]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    net = S.UNet_B("RGB", selective=True, compute_dtype=torch.bfloat16)
    p = L.seeded_params(0, "RGB", True, bn_affine_random=False)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.cuda().train()
    opt = S.Adam(net.parameters(), lr=1e-3)
    loss_a = S.BCEWithLogitsLoss()
    x, lab = make_batch(a.batch, 256, seed=0)
    xt, lt = torch.tensor(x, device="cuda"), torch.tensor(lab, device="cuda")

    def step():
        o, s, au = net(xt)
        loss = loss_a(au, lt) + S.calc_selective_risk_image_b(o, s, target=lt, lamb=2)[0]
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_host = (time.perf_counter() - t0) / a.steps
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / a.steps
    print(f"batch {a.batch}: host enqueue {t_host * 1e3:.2f} ms/step, wall {t_all * 1e3:.2f} ms/step "
          f"-> {a.batch / t_all:.0f} img/s")


if __name__ == "__main__":
    main()
