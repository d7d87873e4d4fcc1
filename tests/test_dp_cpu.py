"""Data-parallel path on CPU: world_size-2 `gloo` process groups exercising `parallel.py`.

The MI355X path replaces DataParallel (train.py:131-134) by one process per GPU. Its exchange
steps are: an all-reduce of the loss partial sums (so every rank computes the
global-batch loss and back-propagates its own pixels with the global normalisers) and a SUM
all-reduce of the flat gradient buffer. This file checks, without a GPU:

* `chunk_bounds` reproduces DataParallel's scatter (torch.chunk) for even, ragged and short
  batches;
* `allreduce_grads` / `allreduce_sums` / `broadcast_params` over a real 2-rank gloo group;
* the sharded-loss decomposition the HIP loss kernels implement: each rank forms the partial
  sums (sum s, sum ell*s, sum bce, pixel count) of its chunk, the sums are all-reduced, and the
  local backward uses d loss / d partial evaluated at the global sums. Run through the oracle
  model on 2 ranks, the summed gradients, the global loss and rank 0's BN buffers equal the
  single-process DataParallel semantics (oracle.train_step(dp_chunks=2)), which
  tests/test_oracle.py pins to the reference's own DataParallel fixture.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from selectivenet_for_semantic_segmentation_binary_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    r, w = parallel.init_data_parallel("gloo")
    assert (r, w) == (rank, world) and parallel.is_initialized()


def _spawn(fn, world, *args):
    mp.spawn(fn, args=(world, _free_port()) + args, nprocs=world, join=True)


@pytest.mark.parametrize("batch,world", [(128, 2), (128, 8), (5, 2), (5, 4), (3, 4), (1, 2), (7, 3)])
def test_chunk_bounds_match_dataparallel_scatter(batch, world):
    x = torch.arange(batch)
    chunks = list(torch.chunk(x, world))
    for r in range(world):
        lo, hi = parallel.chunk_bounds(batch, r, world)
        want = chunks[r].tolist() if r < len(chunks) else []
        assert x[lo:hi].tolist() == want
        assert parallel.local_batch(x, r, world).tolist() == want


# ----------------------------------------------------------------------------- collectives
def _collectives_worker(rank, world, port, out):
    _init(rank, world, port)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    parallel.allreduce_grads(g, bucket_elems=3)  # 4 buckets, the last one ragged
    s = torch.tensor([rank + 0.5, 2.0 * rank], dtype=torch.float64)
    parallel.allreduce_sums(s)
    m = torch.nn.Sequential(torch.nn.Conv2d(2, 3, 3), torch.nn.BatchNorm2d(3))
    with torch.no_grad():
        for p in m.parameters():
            p.fill_(float(rank + 7))
        m[1].running_mean.fill_(float(rank))
    parallel.broadcast_params(m)
    torch.save({"g": g, "s": s, "p": [p.detach().clone() for p in m.parameters()],
                "rm": m[1].running_mean.clone()}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()
    parallel.disable()


def test_collectives_gloo_world2(tmp_path):
    _spawn(_collectives_worker, 2, str(tmp_path))
    ref_g = torch.arange(10, dtype=torch.float32) * 3
    for r in range(2):
        d = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.equal(d["g"], ref_g)
        assert torch.equal(d["s"], torch.tensor([2.0, 2.0], dtype=torch.float64))
        assert all(torch.all(p == 7.0) for p in d["p"])  # rank 0's parameters everywhere
        assert torch.all(d["rm"] == 0.0)


def test_disabled_parallel_is_identity():
    parallel.disable()
    t = torch.ones(3)
    assert parallel.allreduce_grads(t) is t and torch.equal(t, torch.ones(3))
    assert parallel.world_size() == 1 and parallel.rank() == 0


# ----------------------------------------------------------------------------- sharded loss
N, SIZE, LAMB, TARGET_COV = 4, 16, 8.0, 0.8


def _batch():
    from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch
    x, lab = make_batch(N, SIZE, seed=11)
    return torch.tensor(x), torch.tensor(lab)


def _sharded_step_worker(rank, world, port, out):
    """One selective training step as the MI355X ranks compute it, on the oracle model."""
    import torch.nn.functional as F

    from oracle import unet_b_cpu as O
    _init(rank, world, port)
    torch.manual_seed(0)
    params, buffers = O.make_state(seed=3, selective=True)
    x, lab = _batch()
    lo, hi = parallel.chunk_bounds(N, rank, world)
    out_l, sel_l, aux_l = O.forward(params, buffers, x[lo:hi], True, training=True)
    t = lab[lo:hi]
    s = torch.sigmoid(sel_l)
    ell = t * F.softplus(-out_l) + (1 - t) * F.softplus(out_l)
    bce = F.binary_cross_entropy_with_logits(aux_l, t, reduction="sum")
    local = torch.stack([s.sum(), (ell * s).sum(), bce]).double()
    # forward exchange: partial sums + pixel count (selective_loss.py _reduced_sums / global_count)
    sums = parallel.allreduce_sums(torch.cat([local.detach(), torch.tensor([float(out_l.numel())],
                                                                           dtype=torch.float64)]))
    s0, s1, sb, p = sums.tolist()
    cov = s0 / p
    d = max(TARGET_COV - cov, 0.0)
    loss = sb / p + s1 / s0 + LAMB * d * d
    # local backward with the global normalisers (what selunet_selective_bwd / bce_bwd evaluate)
    coef = torch.tensor([-s1 / (s0 * s0) - 2.0 * LAMB * d / p, 1.0 / s0, 1.0 / p], dtype=torch.float64)
    (local * coef).sum().backward()
    names = list(params)
    flat = torch.cat([params[k].grad.reshape(-1) for k in names])
    parallel.allreduce_grads(flat, bucket_elems=1 << 20)
    torch.save({"loss": loss, "coverage": cov, "flat": flat, "names": names,
                "buffers": {k: v.clone() for k, v in buffers.items()}}, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()
    parallel.disable()


@pytest.mark.slow
def test_sharded_selective_loss_equals_dataparallel(tmp_path):
    from oracle import unet_b_cpu as O
    _spawn(_sharded_step_worker, 2, str(tmp_path))
    torch.manual_seed(0)
    params, buffers = O.make_state(seed=3, selective=True)
    opt = O.AdamRef(params.values())
    x, lab = _batch()
    ref = O.train_step(params, buffers, opt, x, lab, True, lamb=int(LAMB), dp_chunks=2)
    ref_flat = torch.cat([g.reshape(-1) for g in ref["grads"].values()])
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["names"] == list(ref["grads"])
    assert abs(r0["loss"] - float(ref["loss"])) < 1e-5 * max(1.0, abs(float(ref["loss"])))
    assert abs(r0["coverage"] - float(ref["coverage"])) < 1e-6
    assert r0["loss"] == r1["loss"]  # every rank sees the global loss
    assert torch.equal(r0["flat"], r1["flat"])  # and the same summed gradient
    scale = ref_flat.abs().max()
    err = (r0["flat"] - ref_flat).abs().max() / scale
    assert err < 1e-5, err
    # replica-0 BN buffers are the ones DataParallel keeps
    for k, v in r0["buffers"].items():
        np.testing.assert_allclose(v.numpy(), buffers[k].detach().numpy(), rtol=1e-5, atol=1e-6, err_msg=k)


# ----------------------------------------------------------------------------- overlapped buckets
def _bucketer_worker(rank, world, port, out):
    _init(rank, world, port)
    import selectivenet_for_semantic_segmentation_binary_amd.layout as L
    specs = L.param_specs("RGB", True)
    names = [k for k, _, _, _ in specs]
    shapes = {k: shp for k, shp, _, _ in specs}
    layout, off = [], 0
    for n in names:
        k = int(np.prod(shapes[n]))
        layout.append((n, off, k))
        off += k
    g = torch.Generator().manual_seed(100 + rank)
    flat = torch.randn(off, generator=g)
    want = flat.clone()
    dist.all_reduce(want)
    b = parallel.GradBucketer(flat, layout, bucket_elems=1 << 18)
    assert len(b.buckets) > 4
    # the engine's backward order: heads, decoder 1_1 ... 4_2, encoder 3_2 ... 1_1
    order = ["heads", "decoder_layer_1_1", "decoder_layer_1_2", "unpool1", "decoder_layer_2_1",
             "decoder_layer_2_2", "unpool2", "decoder_layer_3_1", "decoder_layer_3_2", "unpool3",
             "decoder_layer_4_1", "decoder_layer_4_2", "encoder_layer_3_2", "encoder_layer_3_1",
             "encoder_layer_2_2", "encoder_layer_2_1", "encoder_layer_1_2", "encoder_layer_1_1"]
    assert set(order) == {parallel.grad_layer(n) for n in names}
    launched_before_last = None
    for i, layer in enumerate(order):
        b.ready(layer)
        if i == len(order) - 2:
            launched_before_last = sum(b.launched)
    b.finish()
    out[rank] = (float((flat - want).abs().max()), launched_before_last, len(b.buckets))


def test_grad_bucketer_overlapped_allreduce():
    """Buckets close in backward order (all but the encoder_layer_1_1 one are issued before the last
    layer reports) and the bucketed sum equals one all-reduce of the whole buffer."""
    world = 2
    out = mp.Manager().dict()
    _spawn(_bucketer_worker, world, out)
    for r in range(world):
        err, before_last, nb = out[r]
        assert err < 1e-5
        assert before_last == nb - 1


def _cache_worker(rank, world, port, root, out):
    _init(rank, world, port)
    from selectivenet_for_semantic_segmentation_binary_amd import data as D

    tr, _ = D.construct_train_valid(root, test_fold=5)
    ps = D.decode_patch_list(root, tr, patch_mag=200, patch_size=32, cache=True)
    np.save(os.path.join(out, f"img{rank}.npy"), np.asarray(ps.images))
    dist.destroy_process_group()
    parallel.disable()


def test_patch_cache_shared_by_ranks_without_a_collective(tmp_path):
    """data.decode_patch_list under data parallelism (world 2, gloo): rank 0 decodes and writes the
    uint8 cache, rank 1 waits for the atomically renamed files (no barrier) and maps the same data."""
    from tests._patchdir import make_patch_dir

    root = make_patch_dir(str(tmp_path / "patches"))
    out = tmp_path / "out"
    out.mkdir()
    _spawn(_cache_worker, 2, root, str(out))
    a, b = np.load(out / "img0.npy"), np.load(out / "img1.npy")
    assert a.shape[0] > 0 and np.array_equal(a, b)
