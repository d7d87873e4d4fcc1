"""fp64 gradient truth at the benchmarked shape (BASELINE config 3: SelectiveUNet_B, s_lamb=2, batch 128,
256x256) — test infrastructure, run ON THE GPU BOX:

    python tests/golden/make_truth64.py [--out gpurun_out/truth64_sel_n128_256.npz]

The reference itself cannot run there (it never travels) and its fp64 step at this batch needs ~170 GB,
more than the build container has; so the truth is the oracle's restatement of the reference step
(oracle/unet_b_cpu.py: model.py / selective_loss.py / train.py:194-209) in float64 on the GPU (torch's
own fp64 kernels — the checker, not the product). The oracle is pinned against the reference's fp64
steps at batch 16 (256x256) and batch 2 (512x512) by tests/test_oracle.py.

Writes, for step 0 of step_sel_n128_256.npz's configuration (same seeds, same batch):
  s0/loss64, s0/grad64norm/<name>, the fp64 gradient at the fixture's sampled indices
  (s0/grad64val/<name>, s0/gradidx copied) or in full (s0/grad64full/<name>) as the fixture stores
  it, and s0/grad64proj/<name>: its projections on PROJ seeded Gaussian directions (a whole-tensor
  relative error estimate: tests/test_gpu_fullsize.py regenerates the directions on the GPU)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import unet_b_cpu as O  # noqa: E402  (test infrastructure: the checker)
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402

FIXTURE = os.path.join(REPO, "tests", "golden", "step_sel_n128_256.npz")
PROJ = 16


def directions(name_index, numel, device):
    """PROJ seeded Gaussian directions for tensor number `name_index` (regenerated identically by the test)."""
    g = torch.Generator(device=device)
    g.manual_seed(1000 + name_index)
    return torch.randn(PROJ, numel, generator=g, device=device, dtype=torch.float64)


def project(grads_by_name, names, device):
    out = {}
    for i, k in enumerate(names):
        v = grads_by_name[k].reshape(-1).to(device=device, dtype=torch.float64)
        out[k] = (directions(i, v.numel(), device) @ v).cpu().numpy()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "truth64_sel_n128_256.npz"))
    ap.add_argument("--dry-n", type=int, default=0, help="(script check only: a smaller batch, on the CPU)")
    a = ap.parse_args()
    d = np.load(FIXTURE, allow_pickle=False)
    n, size, lamb = int(d["meta_n"]), int(d["meta_size"]), int(d["meta_lamb"])
    assert bool(d["meta_selective"]) and int(d["meta_chunks"]) == 1
    dev = torch.device("cpu" if a.dry_n else "cuda")
    if a.dry_n:
        n = a.dry_n
    t0 = time.time()
    x, lab = make_batch(n, size, seed=int(d["meta_data_seed"]))
    params, buffers = O.make_state(int(d["meta_seed"]), "RGB", selective=True)
    params = type(params)((k, v.detach().to(dev, torch.float64).requires_grad_()) for k, v in params.items())
    buffers = {k: (v.to(dev, torch.float64) if v.is_floating_point() else v.to(dev)) for k, v in buffers.items()}
    xt = torch.tensor(x, dtype=torch.float64, device=dev)
    lt = torch.tensor(lab, dtype=torch.float64, device=dev)
    del x, lab
    opt = O.AdamRef(params.values(), lr=1e-3)
    print(f"state on device {time.time() - t0:.1f} s", flush=True)
    r = O.train_step(params, buffers, opt, xt, lt, selective=True, lamb=lamb)
    peak = torch.cuda.max_memory_allocated() / 1e9 if dev.type == "cuda" else 0.0
    print(f"fp64 step {time.time() - t0:.1f} s, loss {r['loss'].item():.12g}, peak {peak:.1f} GB", flush=True)
    out = {"meta_source": np.bytes_("oracle/unet_b_cpu.py train_step in float64 on the GPU"),
           "meta_proj": PROJ, "s0/loss64": np.float64(r["loss"].item())}
    names = list(r["grads"].keys())
    out["meta_names"] = np.array(names)
    for k, g in r["grads"].items():
        a64 = g.detach().double().cpu().numpy().ravel()
        out[f"s0/grad64norm/{k}"] = np.float64(np.linalg.norm(a64))
        if f"s0/gradidx/{k}" in d.files:
            idx = d[f"s0/gradidx/{k}"]
            out[f"s0/gradidx/{k}"] = idx
            out[f"s0/grad64val/{k}"] = a64[idx]
        else:
            out[f"s0/grad64full/{k}"] = a64
    for k, p in project(r["grads"], names, dev).items():
        out[f"s0/grad64proj/{k}"] = p
    # the reference's own fp32 step (the fixture) against this truth, for the record
    worst = 0.0
    for k in names:
        ref = d[(f"s0/gradval/{k}" if f"s0/gradidx/{k}" in d.files else f"s0/gradfull/{k}")].astype(np.float64)
        tru = out.get(f"s0/grad64val/{k}", out.get(f"s0/grad64full/{k}"))
        e = float(np.linalg.norm(ref - tru) / max(np.linalg.norm(tru), 1e-30))
        out[f"s0/ref32err/{k}"] = np.float64(e)
        if ".0.bias" not in k or not k.startswith(("encoder", "decoder")):  # (pre-BN conv biases: truth ~0)
            worst = max(worst, e)
    print(f"reference fp32 (fixture) vs fp64 truth: worst relative L2 {worst:.3e} (pre-BN biases aside)", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez_compressed(a.out, **out)
    print(f"wrote {a.out} in {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
