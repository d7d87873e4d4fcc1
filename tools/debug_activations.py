"""Per-layer forward parity of the MI355X path against the fp64 and fp32 oracle (debugging tool).

    python tools/debug_activations.py [--n 2 --size 64 --seed 5 --ce]

For every CBR block: relative max error of the post-BN+ReLU activation, of the BN batch mean and
invstd, and the number of ReLU-mask elements (pre-activation sign) that differ from the fp64
run — for the HIP path and for the fp32 oracle. A kernel that loses precision shows up as a layer
whose error jumps above the oracle's. Test infrastructure only.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from oracle import unet_b_cpu as O  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402


def oracle_acts(x, dt, n_cls):
    params, buffers = O.make_state(0, "RGB", True, n_cls=n_cls)
    params = {k: v.detach().to(dt) for k, v in params.items()}
    buffers = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in buffers.items()}
    acts = {}
    orig = O._cbr

    def cap(p, b, name, t, training):
        y = torch.nn.functional.conv2d(t, p[f"{name}.0.weight"], p[f"{name}.0.bias"], padding=1)
        dims = (0, 2, 3)
        mean = y.mean(dims)
        var = y.var(dims, unbiased=False)
        pre = (y - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + O.BN_EPS)
        pre = pre * p[f"{name}.1.weight"].view(1, -1, 1, 1) + p[f"{name}.1.bias"].view(1, -1, 1, 1)
        acts[name] = (pre, mean - p[f"{name}.0.bias"], 1 / torch.sqrt(var + O.BN_EPS))
        return orig(p, b, name, t, training)

    O._cbr = cap
    try:
        with torch.no_grad():
            O.forward(params, buffers, torch.tensor(x, dtype=dt), True, training=True, ce=n_cls is not None)
    finally:
        O._cbr = orig
    return acts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--ce", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(16)
    x, _ = make_batch(a.n, a.size, seed=a.seed)
    n_cls = 2 if a.ce else None
    a64, a32 = oracle_acts(x, torch.float64, n_cls), oracle_acts(x, torch.float32, n_cls)
    net = (S.UNet("RGB", 2, selective=True) if a.ce else S.UNet_B("RGB", selective=True))
    p = L.seeded_params(0, "RGB", True, n_cls=n_cls)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.cuda().train()
    eng = net._engine()
    P = dict(zip(net._param_names, [t for _, t in net.named_parameters()]))
    B = dict(net.named_buffers())
    xt = torch.tensor(x, device="cuda")
    with torch.no_grad():
        _, ctx = eng.forward(xt, P, B, True, True, need_backward=False, ce_heads=net._ce_heads)
    torch.cuda.synchronize()
    print(f"{'layer':22s} {'ours act':>9s} {'o32 act':>9s} {'ours mean':>9s} {'o32 mean':>9s} {'ours inv':>9s} "
          f"{'o32 inv':>9s} {'ours flips':>10s} {'o32 flips':>9s}")
    for name, _, _ in L.CBR_LAYERS:
        st = ctx.bn[name]
        y = st.y.float().view(st.n, st.h, st.w, st.c).permute(0, 3, 1, 2).cpu().double()
        pre = y * st.scale.cpu().double().view(1, -1, 1, 1) + st.shift.cpu().double().view(1, -1, 1, 1)
        ref_pre, ref_mean, ref_inv = a64[name]
        o_pre, o_mean, o_inv = a32[name]
        scale = ref_pre.abs().max().item()

        def err(t):
            return (torch.relu(t.double()) - torch.relu(ref_pre)).abs().max().item() / scale

        def flips(t):
            return int(((t.double() > 0) != (ref_pre > 0)).sum())

        em = (st.mean.cpu().double() - ref_mean).abs().max().item() / ref_mean.abs().max().item()
        eo = (o_mean.double() - ref_mean).abs().max().item() / ref_mean.abs().max().item()
        ei = ((st.invstd.cpu().double() - ref_inv).abs() / ref_inv).max().item()
        eio = ((o_inv.double() - ref_inv).abs() / ref_inv).max().item()
        print(f"{name:22s} {err(pre):9.2e} {err(o_pre):9.2e} {em:9.2e} {eo:9.2e} {ei:9.2e} {eio:9.2e} "
              f"{flips(pre):10d} {flips(o_pre):9d}")


if __name__ == "__main__":
    main()
