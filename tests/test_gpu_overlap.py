"""The one-GPU all-reduce stand-in (parallel.OverlapEmulation, selunet_cu_hold).

tools/overlap_emulation.py measures how much a CU-holding kernel issued at GradBucketer's bucket
points stretches the backward. These tests pin what that measurement relies on: the stand-in runs
at every bucket point, leaves the gradients bit-identical (it reduce-copies into scratch, never into
the gradient buffer), and the compute stream waits for it before the optimizer reads the gradients.
"""
import numpy as np
import pytest
import torch

import selectivenet_for_semantic_segmentation_binary_amd as S
import selectivenet_for_semantic_segmentation_binary_amd.layout as L
from selectivenet_for_semantic_segmentation_binary_amd import _lib as K
from selectivenet_for_semantic_segmentation_binary_amd import parallel
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grads(emu, bucket_elems=1 << 18):
    x, lab = make_batch(2, 64, seed=3)
    xt, lt = torch.tensor(x, device=DEV), torch.tensor(lab, device=DEV)
    net = S.UNet_B("RGB", selective=True)
    p = L.seeded_params(0, "RGB", True)
    with torch.no_grad():
        for k, t in net.named_parameters():
            t.copy_(torch.tensor(p[k]))
    net = net.to(DEV).train()
    parallel.set_bucket_elems(bucket_elems)
    parallel.set_overlap_emulation(emu)
    try:
        out, sel, aux = net(xt)
        loss = S.BCEWithLogitsLoss()(aux, lt) + S.calc_selective_risk_image_b(out, sel, target=lt, lamb=2)[0]
        loss.backward()
        # read on the compute stream with no extra synchronisation: finish() made it wait on the side stream
        g = torch.cat([q.grad.reshape(-1) for q in net.parameters()]).cpu().numpy()
    finally:
        parallel.set_overlap_emulation(None)
        parallel.set_bucket_elems(1 << 20)
    return g


def test_standin_keeps_gradients_and_runs_at_every_bucket():
    ref = _grads(None)
    emu = parallel.OverlapEmulation(16, 50.0, timing=True)
    got = _grads(emu)
    assert np.array_equal(ref, got)
    n_params = L.count_params("RGB", True)
    assert ref.size == n_params
    # one stand-in per bucket; buckets cover the whole buffer
    assert len(emu.events) >= 2
    assert sum(n for n, _, _ in emu.events) == n_params
    torch.cuda.synchronize()
    for _, e0, e1 in emu.events:
        assert e0.elapsed_time(e1) >= 0.045  # held for its 50 us of wall clock (ms)


def test_cu_hold_argument_checks():
    buf = torch.zeros(64, device=DEV)
    with pytest.raises(K.SelunetError):
        K.call("selunet_cu_hold", K.ptr(buf), K.ptr(buf), 63, 4, 10.0, K.stream_ptr())
    with pytest.raises(K.SelunetError):
        K.call("selunet_cu_hold", K.ptr(buf), K.ptr(buf), 64, 0, 10.0, K.stream_ptr())
