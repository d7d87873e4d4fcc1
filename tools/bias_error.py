"""Where does decoder_layer_4_2.1.bias's gradient error come from? (GPU, study tool)

At the benchmarked shape (batch 128, 256x256, the step_sel_n128_256 fixture's seeds) the HIP fp32
step's worst gradient against fp64 is decoder_layer_4_2's BN beta gradient, 1.33x the reference fp32
step's own error, on both fp32 conv paths. That gradient is sum over pixels of da = dA * relu'(bn(y)),
formed from the BN-backward sums the data gradient of decoder_layer_4_1 accumulates in its epilogue
(model.py:87-88: decoder_layer_4_2 is the first bottleneck block, 4_1 the second). This tool runs
  * the oracle (oracle/unet_b_cpu.py, the checker) in fp64 on the GPU with the CBR outputs' gradients
    retained: the truth dA and the truth beta gradient;
  * the engine's step with dA of decoder_layer_4_2 captured (SELUNET_NO_PLANS=1, a wrapper around
    Engine._cbr_bwd), and its beta gradient;
and prints the relative errors of: the engine's dA (masked) against fp64, the engine's beta gradient,
and the fp64 sum of the engine's own captured da — so the summation (epilogue partial sums, slab
reduction) is separated from the error of the dA values it sums. It repeats the split at every CBR
block, so the layer is seen next to the others.

    SELUNET_NO_PLANS=1 python tools/bias_error.py [--n 128]
"""
import argparse
import os
import sys

os.environ["SELUNET_NO_PLANS"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd import engine as E  # noqa: E402
from oracle import unet_b_cpu as O  # noqa: E402  (the checker)
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402


def rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _heartbeat(period=30.0):
    """A progress line every `period` seconds (a long silent phase would look hung to the GPU harness)."""
    import threading
    import time

    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"  ... {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--data-seed", type=int, default=-1, help="-1: the step_sel_n128_256 fixture's")
    a = ap.parse_args()
    data_seed = a.data_seed
    if data_seed < 0:
        d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                 "step_sel_n128_256.npz"), allow_pickle=False)
        data_seed = int(d["meta_data_seed"])
    dev = torch.device("cuda")
    x, lab = make_batch(a.n, a.size, seed=data_seed)
    layers = [nm for nm, _, _ in L.CBR_LAYERS]

    # ---- ours: capture dA of every CBR block and its BN state
    cap = {}
    orig = E.Engine._cbr_bwd

    def wrapped(self, ctx, name, dg, G, input_srcs, **kw):
        st = ctx.bn[name]
        if dg.t is not None:
            cap[name] = (dg.t.detach().clone(), st.y.detach().clone(), st.scale.clone(), st.shift.clone())
        else:  # producer in sums-only mode (heads / pools): dA is formed inside the apply, not stored
            cap[name] = None
        return orig(self, ctx, name, dg, G, input_srcs, **kw)

    E.Engine._cbr_bwd = wrapped
    net = S.UNet_B("RGB", selective=True)
    p = L.seeded_params(a.seed, "RGB", True)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(dev).train()
    xt, lt = torch.tensor(x, device=dev), torch.tensor(lab, device=dev)
    out, sel, aux = net(xt)
    loss = S.BCEWithLogitsLoss()(aux, lt) + S.calc_selective_risk_image_b(out, sel, target=lt, lamb=2)[0]
    loss.backward()
    torch.cuda.synchronize()
    ours_g = {k: q.grad.detach().double().cpu() for k, q in net.named_parameters()}
    E.Engine._cbr_bwd = orig
    print("engine step done", flush=True)
    del net, out, sel, aux, loss
    torch.cuda.empty_cache()

    # ---- fp64 oracle with every CBR output's gradient retained
    zs = {}
    ocbr = O._cbr

    def rec(params, buffers, name, t, training):
        z = ocbr(params, buffers, name, t, training)
        z.retain_grad()
        zs[name] = z
        return z

    O._cbr = rec
    params, buffers = O.make_state(a.seed, "RGB", selective=True)
    params = type(params)((k, v.detach().to(dev, torch.float64).requires_grad_()) for k, v in params.items())
    buffers = {k: (v.to(dev, torch.float64) if v.is_floating_point() else v.to(dev)) for k, v in buffers.items()}
    opt = O.AdamRef(params.values(), lr=1e-3)
    r = O.train_step(params, buffers, opt, torch.tensor(x, dtype=torch.float64, device=dev),
                     torch.tensor(lab, dtype=torch.float64, device=dev), selective=True, lamb=2)
    r_loss = float(r["loss"])
    O._cbr = ocbr
    g64 = {k: v.detach().double().cpu() for k, v in r["grads"].items()}
    da64s, mask64s = {}, {}
    for nm in layers:
        z = zs[nm]
        mask64s[nm] = (z.detach() > 0).permute(0, 2, 3, 1).reshape(-1, z.shape[1])
        da64s[nm] = (z.grad.detach() * (z.detach() > 0)).permute(0, 2, 3, 1).reshape(-1, z.shape[1])
    del zs, r, params, buffers, opt
    torch.cuda.empty_cache()
    print("fp64 oracle step done", flush=True)

    # ---- the same oracle in fp32 (torch's own GPU kernels: a third fp32 implementation of the reference step)
    zs32 = {}

    def rec32(params, buffers, name, t, training):
        z = ocbr(params, buffers, name, t, training)
        z.retain_grad()
        zs32[name] = z
        return z

    O._cbr = rec32
    # torch's native convolutions (im2col + BLAS), not MIOpen: no kernel compilation / search on a fresh box
    torch.backends.cudnn.enabled = False
    p32, b32 = O.make_state(a.seed, "RGB", selective=True)
    p32 = type(p32)((k, v.detach().to(dev, torch.float32).requires_grad_()) for k, v in p32.items())
    b32 = {k: (v.to(dev, torch.float32) if v.is_floating_point() else v.to(dev)) for k, v in b32.items()}
    r32 = O.train_step(p32, b32, O.AdamRef(p32.values(), lr=1e-3), torch.tensor(x, device=dev),
                       torch.tensor(lab, device=dev), selective=True, lamb=2)
    O._cbr = ocbr
    g32 = {k: v.detach().double().cpu() for k, v in r32["grads"].items()}
    print("fp32 oracle step done", flush=True)

    print(f"loss (fp64) {float(r_loss):.9f}", flush=True)
    print("per CBR block: relative L2 error against the fp64 oracle of dA (masked: da = dA relu'), of the BN beta\n"
          "gradient (= sum of da), of the fp64 sum of the engine's own da (the summation's share), the number of\n"
          "ReLU-mask flips, and the dA error without the flipped pixels; the same for torch-fp32 (the oracle on the GPU)")
    print(f"{'layer':22s} {'dA err':>9s} {'beta err':>9s} {'sum(own)':>9s} {'flips':>8s} {'dA err nf':>9s} | "
          f"{'fp32 dA':>9s} {'fp32 beta':>9s} {'flips':>8s} {'dA err nf':>9s} | {'|sum da|/sum|da|':>16s}")
    for nm in layers:
        da64, m64 = da64s[nm], mask64s[nm]
        beta64 = g64[f"{nm}.1.bias"]
        cancel = float(beta64.abs().sum() / da64.abs().sum(0).sum().cpu())
        eb = rel(ours_g[f"{nm}.1.bias"], beta64)
        z32 = zs32[nm]
        m32 = (z32.detach() > 0).permute(0, 2, 3, 1).reshape(-1, z32.shape[1])
        da32 = (z32.grad.detach() * (z32.detach() > 0)).permute(0, 2, 3, 1).reshape(-1, z32.shape[1]).double()
        f32 = m32 != m64
        e32, eb32, nf32 = rel(da32, da64), rel(g32[f"{nm}.1.bias"], beta64), int(f32.sum())
        e32nf = rel(da32[~f32], da64[~f32])
        if cap.get(nm) is None:
            print(f"{nm:22s} {'(fused)':>9s} {eb:9.2e} {'-':>9s} {'-':>8s} {'-':>9s} | {e32:9.2e} {eb32:9.2e} "
                  f"{nf32:8d} {e32nf:9.2e} | {cancel:16.2e}", flush=True)
            continue
        dA, y, sc, sh = cap[nm]
        mask = (y * sc + sh) > 0
        da = dA.double() * mask
        fl = mask != m64
        e_da, e_sum, nfl = rel(da, da64), rel(da.sum(0).cpu(), beta64), int(fl.sum())
        e_nf = rel(da[~fl], da64[~fl])
        print(f"{nm:22s} {e_da:9.2e} {eb:9.2e} {e_sum:9.2e} {nfl:8d} {e_nf:9.2e} | {e32:9.2e} {eb32:9.2e} "
              f"{nf32:8d} {e32nf:9.2e} | {cancel:16.2e}", flush=True)
        del dA, y, da


if __name__ == "__main__":
    main()
