"""One rank of the multi-process data-parallel GPU test (tests/test_gpu_dp.py).

Runs the golden fixture's training steps exactly as a `--gpus N` job would (train.py:186-209
with DataParallel replaced by one process per rank): the rank takes its contiguous chunk of the
batch, runs the MI355X UNet_B / selective loss / BCE / Adam, with the loss partial sums and the
gradients all-reduced by `parallel`. Rank r writes its results to OUT/r{r}_s{step}.npz.
Backend "gloo": all ranks share cuda:0 (one-GPU box). Backend "nccl" (RCCL over xGMI): rank r
runs on cuda:r, as `bench.py --gpus N` and `train.py --local_rank ...` do.
"""
import os
import sys

import numpy as np
import torch

import selectivenet_for_semantic_segmentation_binary_amd as S
from selectivenet_for_semantic_segmentation_binary_amd import parallel
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch
from tests import _golden as G
from tests.test_gpu_model import build


def main(fname, out, backend="gloo"):
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local if backend == "nccl" else 0)
    rank, world = parallel.init_data_parallel(backend)
    d = G.load(fname)
    n, size, selective = int(d["meta_n"]), int(d["meta_size"]), bool(d["meta_selective"])
    assert world == int(d["meta_chunks"]), (world, int(d["meta_chunks"]))
    x, lab = make_batch(n, size, seed=int(d["meta_data_seed"]))
    lo, hi = parallel.chunk_bounds(n, rank, world)
    parallel.set_global_batch(n)
    xt = torch.tensor(x[lo:hi], device="cuda")
    lt = torch.tensor(lab[lo:hi], device="cuda")
    net = build(selective, int(d["meta_seed"]))
    parallel.broadcast_params(net)
    opt = S.Adam(net.parameters(), lr=1e-3)
    loss_A = S.BCEWithLogitsLoss()
    for s in range(int(d["meta_steps"])):
        o, sel, aux = net(xt)
        aux_loss = loss_A(aux, lt)
        select_loss, coverage = S.calc_selective_risk_image_b(o, sel, target=lt, lamb=int(d["meta_lamb"]))
        loss = aux_loss + select_loss
        opt.zero_grad()
        loss.backward()
        res = {"world": torch.distributed.get_world_size(), "backend": torch.distributed.get_backend(),
               "loss": loss.item(), "coverage": coverage.item(), "aux_loss": aux_loss.item(),
               "select_loss": select_loss.item(), "output": o.detach().cpu().numpy(),
               "selection": sel.detach().cpu().numpy(), "aux": aux.detach().cpu().numpy()}
        if rank == 0:
            for k, p in net.named_parameters():
                res["grad/" + k] = p.grad.detach().cpu().numpy()
        opt.step()
        if rank == 0:
            for k, p in net.named_parameters():
                res["param/" + k] = p.detach().cpu().numpy()
            for k, v in net.named_buffers():
                res["buf/" + k] = v.cpu().numpy()
        np.savez(os.path.join(out, f"r{rank}_s{s}.npz"), **res)
    torch.cuda.synchronize()
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *sys.argv[3:4])
