"""Layer-by-layer backward comparison (dZ entering each CBR block, per DataParallel chunk)
between the MI355X engine and the fp64 oracle. Test infrastructure only.

    python tools/debug_layers.py --n 8 --size 32 --chunks 4
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import engine as E  # noqa: E402
from oracle import unet_b_cpu as O  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--chunks", type=int, default=4)
    a = ap.parse_args()
    x, lab = make_batch(a.n, a.size, seed=1)

    # ---- oracle fp64 with z.retain_grad() on every CBR output
    zs = defaultdict(list)
    orig = O._cbr

    def rec(params, buffers, name, t, training):
        z = orig(params, buffers, name, t, training)
        z.retain_grad()
        zs[name].append(z)
        return z

    O._cbr = rec
    params, buffers = O.make_state(0, "RGB", True)
    for k in params:
        params[k] = params[k].detach().double().requires_grad_()
    for k in buffers:
        if buffers[k].is_floating_point():
            buffers[k] = buffers[k].double()
    opt = O.AdamRef(params.values())
    O.train_step(params, buffers, opt, torch.tensor(x).double(), torch.tensor(lab).double(), True, lamb=2,
                 loss_form="stable", dp_chunks=a.chunks)
    O._cbr = orig

    # ---- ours: record dz entering each _cbr_bwd, keyed by the chunk's input pointer
    got = defaultdict(dict)
    orig_bwd = E.Engine._cbr_bwd

    def rec_bwd(self, ctx, name, dz, G, srcs, **kw):
        st = ctx.bn[name]
        got[name][ctx.x.data_ptr()] = dz.detach().double().cpu().reshape(st.n, st.h, st.w, st.c).permute(0, 3, 1, 2)
        return orig_bwd(self, ctx, name, dz, G, srcs, **kw)

    E.Engine._cbr_bwd = rec_bwd
    net = S.UNet_B("RGB", selective=True)
    p = L.seeded_params(0, "RGB", True)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.cuda().train()
    xt, lt = torch.tensor(x, device="cuda"), torch.tensor(lab, device="cuda")
    chunks = torch.chunk(xt, a.chunks)
    outs = [net(xc) for xc in chunks]
    o, s, au = (torch.cat([q[i] for q in outs]) for i in range(3))
    sl, cov = S.calc_selective_risk_image_b(o, s, lt, lamb=2)
    loss = S.BCEWithLogitsLoss()(au, lt) + sl
    loss.backward()
    torch.cuda.synchronize()
    ptrs = [c.data_ptr() for c in chunks]
    order = [n for n, _, _ in reversed(L.CBR_LAYERS)]
    print(f"{'layer':22s} " + " ".join(f"chunk{r:<6d}" for r in range(a.chunks)))
    for name in order:
        row = []
        for r in range(a.chunks):
            ref = zs[name][r].grad
            mine = got[name].get(ptrs[r])
            if mine is None:
                row.append("   missing")
                continue
            e = float((mine - ref).abs().max() / (ref.abs().max() + 1e-30))
            row.append(f"{e:9.2e}")
        print(f"{name:22s} " + " ".join(row))


if __name__ == "__main__":
    main()
