"""Data parallelism: one process per GPU replacing `torch.nn.DataParallel` (train.py:131-134).

The reference runs single-process DataParallel: the global batch is scattered in contiguous
chunks (torch.chunk semantics), each replica runs BatchNorm on its own chunk, the three head
outputs are gathered to cuda:0 where the selective loss is evaluated on the *global* batch,
gradients are reduce-added to cuda:0, and only replica 0's BN running statistics persist.

Here each rank owns one GPU and one chunk. The exchange steps are exactly the ones the
math needs:
  * forward: all-reduce (sum) of the loss partial sums — 2 doubles for the selective risk
    (sum sigmoid(g), sum ell*sigmoid(g)) + the pixel count, 1 for the aux BCE — so every rank
    sees the global-batch loss and computes its local per-pixel gradients with the global
    normalisers;
  * backward: all-reduce (sum, not mean) of the flat fp32 gradient buffer (30.8 MB);
  * eval: rank 0's BN buffers broadcast before an eval-mode forward (DataParallel re-broadcasts
    device-0 buffers every forward).
Backend "nccl" is RCCL on ROCm (xGMI within a node); "gloo" is used by the CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_STATE = {"enabled": False, "group": None, "global_batch": None, "emulate": None, "bucket_elems": 1 << 20}


def init_data_parallel(backend: str | None = None, group=None) -> tuple[int, int]:
    """Initialise (if needed) the default process group from RANK/WORLD_SIZE/MASTER_* env vars
    and enable the data-parallel exchanges. Returns (rank, world_size)."""
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend)
    _STATE["enabled"] = dist.get_world_size(group) > 1
    _STATE["group"] = group
    return dist.get_rank(group), dist.get_world_size(group)


def disable():
    _STATE["enabled"] = False
    _STATE["group"] = None
    _STATE["global_batch"] = None


def set_global_batch(batch: int | None):
    """Register the global batch size B the ranks' chunks come from (chunk_bounds), so the losses
    know the global pixel count B*H*W without an exchange (selective_loss.global_count)."""
    _STATE["global_batch"] = None if batch is None else int(batch)


def global_batch() -> int | None:
    return _STATE["global_batch"]


def is_initialized() -> bool:
    return _STATE["enabled"] and dist.is_initialized()


class OverlapEmulation:
    """One-GPU stand-in for the bucketed gradient all-reduce (tools/overlap_emulation.py).

    At each point GradBucketer would issue an RCCL all-reduce, a CU-holding reduce-copy kernel
    (`selunet_cu_hold`: n_wg workgroups, `us` microseconds of wall clock each) is launched on a side
    stream that first waits on the compute stream — the stream relationship ProcessGroupNCCL sets
    up — and `finish` makes the compute stream wait for it, as `Work.wait()` does. The kernel reads
    the bucket and reduce-copies into a scratch buffer, so the gradients are untouched. `events`
    collects (bucket elements, start, end) HIP event pairs on the side stream when timing is on."""

    def __init__(self, n_wg: int, us: float, timing: bool = False, model: tuple | None = None, priority: int = 0):
        # model (alpha_us, beta_GBs): hold each bucket's CUs for alpha + bytes / beta instead of `us`;
        # priority: the side stream's (-1 = high, as ProcessGroupNCCL's streams with is_high_priority_stream)
        self.n_wg, self.us, self.timing, self.model = int(n_wg), float(us), timing, model
        self.priority = int(priority)
        self.held_us = 0.0
        self.side = None
        self.scratch = None
        self.events = []

    def launch(self, t: torch.Tensor):
        from . import _lib as K
        if self.side is None:
            self.side = torch.cuda.Stream(device=t.device, priority=self.priority)
        if self.scratch is None or self.scratch.numel() < t.numel() + 4:
            self.scratch = torch.zeros(t.numel() + 4, dtype=torch.float32, device=t.device)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        self.side.wait_event(ev)
        n = (t.numel() // 4) * 4
        if n == 0:  # (a bucket under 4 floats: nothing the 16-B reduce-copy could read in bounds)
            return
        us = self.us if self.model is None else self.model[0] + t.numel() * 4 / (self.model[1] * 1e3)
        self.held_us += us
        with torch.cuda.stream(self.side):
            e0 = e1 = None
            if self.timing:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(self.side)
            K.call("selunet_cu_hold", K.ptr(t), K.ptr(self.scratch), n, self.n_wg, us,
                   self.side.cuda_stream)
            if self.timing:
                e1.record(self.side)
                self.events.append((t.numel(), e0, e1))

    def finish(self, device):
        if self.side is not None:
            torch.cuda.current_stream(device).wait_stream(self.side)


def set_overlap_emulation(emu: "OverlapEmulation | None"):
    """Install (or remove, None) the one-GPU all-reduce stand-in: with it, the backward builds a
    GradBucketer on a single process and launches the stand-in kernel at every bucket point."""
    _STATE["emulate"] = emu


def overlap_emulation() -> "OverlapEmulation | None":
    return _STATE["emulate"]


def set_bucket_elems(n: int):
    """Minimum gradient-bucket size in floats (default 1 << 20 = 4 MB)."""
    _STATE["bucket_elems"] = int(n)


def bucket_elems() -> int:
    return _STATE["bucket_elems"]


def world_size() -> int:
    return dist.get_world_size(_STATE["group"]) if is_initialized() else 1


def rank() -> int:
    return dist.get_rank(_STATE["group"]) if is_initialized() else 0


def allreduce_sums(t: torch.Tensor) -> torch.Tensor:
    """In-place global sum of a small partial-sum vector (loss forward exchange)."""
    if is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=_STATE["group"])
    return t


def allreduce_grads(flat: torch.Tensor, bucket_elems: int = 1 << 22) -> torch.Tensor:
    """Sum replica gradients (DataParallel reduce_add semantics), in buckets."""
    if not is_initialized():
        return flat
    n = flat.numel()
    works = []
    for off in range(0, n, bucket_elems):
        works.append(dist.all_reduce(flat[off:off + bucket_elems], op=dist.ReduceOp.SUM, group=_STATE["group"],
                                     async_op=True))
    for w in works:
        w.wait()
    return flat


def grad_layer(param_name: str) -> str:
    """The engine layer whose backward writes this parameter's gradient (Engine.backward on_grads
    tags): the module prefix, or "heads" for the 1x1 heads (reduced together)."""
    mod = param_name.split(".")[0]
    return "heads" if mod in ("conv1x1", "conv_select", "conv_aux") else mod


class GradBucketer:
    """SUM all-reduce of the flat gradient buffer in buckets overlapped with the backward.

    Buckets are runs of consecutive parameters (flat = registration order) of at least
    `bucket_elems` floats, cut at parameter boundaries and formed from the END of the buffer: the
    backward produces the head and decoder gradients first and encoder_layer_1_1's last. A bucket's
    all-reduce is enqueued (async, RCCL's stream waits on the compute stream up to that point) as
    soon as every layer it covers has reported its gradients through `ready`; `finish` enqueues
    anything left and makes the current stream wait for all of them. Every rank reports the layers
    in the same order, so the collectives are issued in the same order everywhere."""

    def __init__(self, flat: torch.Tensor, layout, bucket_elems: int = 1 << 20, emulate: OverlapEmulation = None):
        # layout: [(param_name, offset, numel)] in flat order
        self.flat = flat
        self.emulate = emulate
        self.buckets = []          # [lo, hi, pending layer set]
        self.works = []
        cur_hi, cur_lo, layers = None, None, set()
        for name, off, n in reversed(list(layout)):
            if cur_hi is None:
                cur_hi = off + n
            cur_lo = off
            layers.add(grad_layer(name))
            if cur_hi - cur_lo >= bucket_elems:
                self.buckets.append([cur_lo, cur_hi, layers])
                cur_hi, layers = None, set()
        if cur_hi is not None:
            self.buckets.append([cur_lo, cur_hi, layers])
        self.launched = [False] * len(self.buckets)

    def _launch(self, i):
        lo, hi, _ = self.buckets[i]
        self.launched[i] = True
        if is_initialized():
            self.works.append(dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=_STATE["group"],
                                              async_op=True))
        elif self.emulate is not None:
            self.emulate.launch(self.flat[lo:hi])

    def ready(self, layer: str):
        for i, b in enumerate(self.buckets):
            if not self.launched[i] and layer in b[2]:
                b[2].discard(layer)
                if not b[2]:
                    self._launch(i)

    def finish(self) -> torch.Tensor:
        for i in range(len(self.buckets)):
            if not self.launched[i]:
                self._launch(i)
        for w in self.works:
            w.wait()
        self.works = []
        if self.emulate is not None:
            self.emulate.finish(self.flat.device)
        return self.flat


def broadcast_buffers(module: torch.nn.Module):
    if not is_initialized():
        return
    for b in module.buffers():
        dist.broadcast(b, src=0, group=_STATE["group"])


def broadcast_params(module: torch.nn.Module):
    """Make every rank start from rank 0's parameters and buffers."""
    if not dist.is_initialized():
        return
    with torch.no_grad():
        for p in module.parameters():
            dist.broadcast(p.data, src=0, group=_STATE["group"])
        for b in module.buffers():
            dist.broadcast(b, src=0, group=_STATE["group"])


def chunk_bounds(batch: int, rank_: int, world: int) -> tuple[int, int]:
    """Rows [lo, hi) of replica `rank_` under DataParallel's scatter (torch.chunk on dim 0:
    chunks of ceil(batch / world), the last ones possibly shorter or empty)."""
    size = -(-batch // world)
    lo = min(batch, rank_ * size)
    hi = min(batch, lo + size)
    return lo, hi


def local_batch(x: torch.Tensor, rank_: int | None = None, world: int | None = None) -> torch.Tensor:
    r = rank() if rank_ is None else rank_
    w = world_size() if world is None else world
    if rank_ is None and world is None:
        set_global_batch(x.shape[0])
    lo, hi = chunk_bounds(x.shape[0], r, w)
    return x[lo:hi]
