"""Multi-process data parallelism on the GPU against the reference's DataParallel fixtures.

N ranks (tests/dp_worker.py, one process each) train on contiguous chunks of the 8-image batch:
over a `gloo` group all on cuda:0 (runs on the one-GPU box), and over RCCL (`nccl`, rank r on
cuda:r — the path bench.py --gpus N and train.py --local_rank take) whenever the box has at
least N GPUs; their concatenated logits, the global
loss/coverage every rank reports, the summed gradients and rank 0's parameters and BN buffers
are compared with `dp_sel_n8_32_c4.npz` — the reference model run under DataParallel-chunk
semantics over 4 replicas (tests/golden/make_golden.py) — with the same checks as the
single-process fixtures (tests/test_gpu_model.py::check_step).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests import _golden as G
from tests.test_gpu_model import check_step

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.parametrize("fname,backend", [
    ("dp_sel_n8_32_c4.npz", "gloo"),
    # the world size train.sh:1 runs (8 device ids), rehearsed with all 8 ranks on cuda:0
    ("dp_sel_n16_32_c8.npz", "gloo"),
    pytest.param("dp_sel_n8_32_c2.npz", "nccl",
                 marks=pytest.mark.skipif(_gpus() < 2, reason="RCCL data parallelism needs >= 2 GPUs")),
    pytest.param("dp_sel_n8_32_c4.npz", "nccl",
                 marks=pytest.mark.skipif(_gpus() < 4, reason="RCCL data parallelism needs >= 4 GPUs")),
    pytest.param("dp_sel_n16_32_c8.npz", "nccl",
                 marks=pytest.mark.skipif(_gpus() < 8, reason="RCCL data parallelism needs >= 8 GPUs")),
])
def test_multi_rank_dp_matches_dataparallel_fixture(fname, backend, tmp_path):
    d = G.load(fname)
    world = int(d["meta_chunks"])
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-m", "tests.dp_worker", fname, str(tmp_path), backend],
                                      cwd=REPO, env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=300))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes
    fails = []
    for s in range(int(d["meta_steps"])):
        rs = [np.load(tmp_path / f"r{r}_s{s}.npz") for r in range(world)]
        # each rank reports the group it ran in: size and backend as torch.distributed saw them
        assert [(int(x["world"]), str(x["backend"])) for x in rs] == [(world, backend)] * world
        losses = {float(x["loss"]) for x in rs}
        assert len(losses) == 1, losses  # every rank computed the same global loss
        r0 = rs[0]
        res = {"loss": float(r0["loss"]), "coverage": float(r0["coverage"]),
               "aux_loss": float(r0["aux_loss"]), "select_loss": float(r0["select_loss"]),
               "output": np.concatenate([x["output"] for x in rs]),
               "selection": np.concatenate([x["selection"] for x in rs]),
               "aux": np.concatenate([x["aux"] for x in rs]),
               "grads": {k[5:]: r0[k] for k in r0.files if k.startswith("grad/")},
               "params": {k[6:]: r0[k] for k in r0.files if k.startswith("param/")},
               "buffers": {k[4:]: r0[k] for k in r0.files if k.startswith("buf/")}}
        res["num_batches_tracked"] = int(res["buffers"]["encoder_layer_1_1.1.num_batches_tracked"])
        fails += check_step(d, s, res, strict=s < 1)
    assert not fails, "\n".join(fails[:25])
