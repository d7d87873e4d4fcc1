"""Patch data for the training loop: pre-decoded uint8 shards on the host,
normalisation / flips / NCHW fp32 conversion on the GPU (`selunet_prep_batch`).

The reference decodes every JPEG/PNG patch with PIL inside `PatchDataset.__getitem__`
(utils/data_utils.py:170-236) and applies `Normalization`, `RandomFlip` and `ToTensor` in numpy on
16 DataLoader workers (train.py:360-380). Here a split is decoded ONCE into a uint8 NHWC array
(an `.npy` cache next to the patches, memory-mapped afterwards), each global batch is gathered
into pinned memory by a prefetch thread, copied to the GPU as uint8 (4x fewer bytes than fp32)
and expanded there. Data-parallel ranks take their contiguous chunk of every global batch
(DataParallel's scatter, parallel.chunk_bounds).

Split construction (`construct_train_valid` / `construct_test`) follows
utils/data_utils.py:49-86, including the module-level `np.random.seed(42)` the reference's
`split_train_valid` draws from (reproduced with a RandomState(42) consumed in the same order).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os

import numpy as np
import torch

from . import _lib as K
from . import parallel
from .synthetic import make_patches


class PatchSet:
    """images uint8 [N,H,W,3] (RGB), labels uint8 [N,H,W] (raw mask values; only 255 is tumor)."""

    def __init__(self, images, labels, ids=None):
        if images.ndim != 4 or images.shape[-1] != 3 or labels.shape != images.shape[:3]:
            raise ValueError(f"PatchSet: images {images.shape} / labels {labels.shape} must be [N,H,W,3] / [N,H,W]")
        if images.dtype != np.uint8 or labels.dtype != np.uint8:
            raise ValueError("PatchSet: images and labels must be uint8")
        self.images, self.labels, self.ids = images, labels, ids

    def __len__(self):
        return self.images.shape[0]

    @property
    def hw(self):
        return self.images.shape[1], self.images.shape[2]


def synthetic_patchset(n: int, size: int = 256, seed: int = 0) -> PatchSet:
    imgs, labs = make_patches(n, size, seed)
    return PatchSet(imgs, labs)


def load_test_set_for_tests(spec: str, size: int, test_fold: int):
    """The synthetic test fold `--data_dir synthetic:N` names: N patches, fold by index (uint8
    images [N,H,W,3], labels [N,H,W])."""
    n = int(spec.split(":")[1]) if ":" in spec else 64
    imgs, labs = make_patches(5 * n, size, seed=1000)
    idx = np.nonzero(np.arange(5 * n) % 5 + 1 == test_fold)[0]
    return imgs[idx], labs[idx]


# ----------------------------------------------------------------------------- split lists
def _split_train_valid(rs, lst, valid_ratio=0.2):
    """utils/data_utils.py:52-56."""
    total_n = len(lst)
    valid_idx = rs.choice(total_n, size=int(total_n * valid_ratio), replace=False)
    train_idx = np.setdiff1d([i for i in range(total_n)], valid_idx)
    return lst[train_idx], lst[valid_idx]


def construct_train_valid(data_dir, test_fold=5):
    """utils/data_utils.py:58-76: folds != test_fold, 20% of each class held out for validation."""
    rs = np.random.RandomState(42)  # utils/data_utils.py:50 (module-level np.random.seed(42))
    folds = [f for f in (1, 2, 3, 4, 5) if f != test_fold]
    tum = np.concatenate([np.load(f"{data_dir}/{i}-fold_tumorable_data.npy") for i in folds])
    non = np.concatenate([np.load(f"{data_dir}/{i}-fold_non_tumorable_data.npy") for i in folds])
    t_train, t_valid = _split_train_valid(rs, tum, 0.2)
    n_train, n_valid = _split_train_valid(rs, non, 0.2)
    return np.vstack([t_train, n_train]), np.vstack([t_valid, n_valid])


def construct_test(data_dir, test_fold=1):
    """utils/data_utils.py:78-86."""
    tum = np.load(f"{data_dir}/{test_fold}-fold_tumorable_data.npy")
    non = np.load(f"{data_dir}/{test_fold}-fold_non_tumorable_data.npy")
    return np.vstack([np.array(tum), np.array(non)])


def decode_patch_list(data_dir, data_list, patch_mag=200, patch_size=256, cache=True) -> PatchSet:
    """Decode (input .jpg, label .png) pairs of `{data_dir}/{patch_mag}x_{patch_size}/` once
    (PIL, as PatchDataset.__getitem__, utils/data_utils.py:209-217) into uint8 arrays; with
    cache=True they are stored as .npy next to the patches and memory-mapped on later runs.

    Under data parallelism (one process per GPU, `train.py --local_rank ...`) only rank 0 decodes:
    it writes each cache file under a temporary name and renames it into place (os.replace is
    atomic, so no rank can map a half-written file) while the other ranks poll for the finished
    files (no collective: a long first decode cannot run into the process group's timeout, and the
    wait does not go through the GPU backend), and every rank then memory-maps the cache — one
    decoded copy on the host instead of one per GPU."""
    from PIL import Image

    root = os.path.join(data_dir, f"{patch_mag}x_{patch_size}")
    pairs = [(str(a), str(b)) for a, b in data_list]
    for a, b in pairs:
        if a.split("_input")[0] != b.split("_label")[0]:
            raise ValueError(f"check the pairness btw input {a} and label {b}")
    key = hashlib.sha1("\n".join(a + "|" + b for a, b in pairs).encode()).hexdigest()[:16]
    cdir = os.path.join(root, "_selunet_cache")
    fi, fl = os.path.join(cdir, f"{key}_images.npy"), os.path.join(cdir, f"{key}_labels.npy")
    ids = [a.split("_input")[0] for a, _ in pairs]
    shared = cache and parallel.is_initialized() and parallel.world_size() > 1
    failed = os.path.join(cdir, f"{key}_FAILED")
    if shared and parallel.rank() != 0:
        # rank 0 writes (or has written) the cache, or leaves the failure marker
        _wait_for_files((fi, fl), CACHE_WAIT_S, failed=failed)
        return PatchSet(np.load(fi, mmap_mode="r"), np.load(fl, mmap_mode="r"), ids)
    if cache and os.path.exists(fi) and os.path.exists(fl):
        return PatchSet(np.load(fi, mmap_mode="r"), np.load(fl, mmap_mode="r"), ids)
    imgs = np.empty((len(pairs), patch_size, patch_size, 3), np.uint8)
    labs = np.empty((len(pairs), patch_size, patch_size), np.uint8)
    if shared and os.path.exists(failed):
        os.remove(failed)
    try:
        for i, (a, b) in enumerate(pairs):
            imgs[i] = np.array(Image.open(os.path.join(root, a)).convert("RGB"))
            labs[i] = np.array(Image.open(os.path.join(root, b)).convert("L"))
        if cache:
            os.makedirs(cdir, exist_ok=True)
            for path, arr in ((fi, imgs), (fl, labs)):
                tmp = f"{path[:-4]}.tmp{os.getpid()}.npy"
                np.save(tmp, arr)
                os.replace(tmp, path)
    except Exception as e:
        if shared:  # the waiting ranks stop at once instead of polling until CACHE_WAIT_S
            os.makedirs(cdir, exist_ok=True)
            with open(failed, "w") as f:
                f.write(f"rank 0 failed to decode or cache the patch list: {e!r}\n")
        raise
    return PatchSet(imgs, labs, ids)


CACHE_WAIT_S = float(os.environ.get("SELUNET_CACHE_WAIT_S", 6 * 3600))


def _process_start_time() -> float:
    """Wall-clock start of this process (psutil), or the import of this module without psutil."""
    try:
        import psutil

        return float(psutil.Process().create_time())
    except Exception:  # pragma: no cover - psutil is part of the image
        return _IMPORT_TIME


_IMPORT_TIME = __import__("time").time()


def _wait_for_files(paths, limit_s, poll_s=0.5, failed=None, since=None):
    """Block until every path exists (they appear atomically, os.replace) or limit_s passes; raise
    as soon as the `failed` marker (written by the rank that was to produce them) appears.

    Only a marker written by this launch counts: one whose mtime is before `since` (default: this
    process's start) is left over from an earlier failed run — every process of a new launch starts
    after the old run ended, while this launch's rank 0 can only fail after the process group's
    rendezvous, i.e. after every rank has started — and is ignored (rank 0 deletes it when it starts
    decoding)."""
    import time

    since = _process_start_time() if since is None else since
    t0 = time.monotonic()
    while not all(os.path.exists(p) for p in paths):
        if failed is not None and os.path.exists(failed):
            try:
                fresh = os.stat(failed).st_mtime >= since
                msg = open(failed).read().strip() if fresh else None
            except OSError:  # removed between the checks (rank 0 clearing a stale marker)
                fresh = False
            if fresh:
                raise RuntimeError(msg)
        if time.monotonic() - t0 > limit_s:
            raise TimeoutError(f"rank 0 did not write the patch cache within {limit_s:.0f} s: {paths}")
        time.sleep(poll_s)


# ----------------------------------------------------------------------------- GPU batches
_CIN = {"RGB": 3, "GH": 2, "H_RGB": 3}
_MODE = {"RGB": 0, "GH": 1, "H_RGB": 2}


def prep_batch(images_u8: torch.Tensor, labels_u8: torch.Tensor, flips: torch.Tensor | None = None,
               input_type: str = "RGB"):
    """uint8 NHWC patches + uint8 masks on the GPU -> (x fp32 [N,C,H,W], target fp32 [N,H,W]),
    the reference's [RGB2GH +] Normalization + RandomFlip + ToTensor + label/255 truncation
    (C = 3 for input_type 'RGB' and 'H_RGB', 2 for 'GH': utils/data_utils.py:13-41, 223-226)."""
    if input_type not in _CIN:
        raise ValueError(f"input_type {input_type!r}: 'RGB', 'GH' or 'H_RGB' (utils/data_utils.py:223-226)")
    for name, t in (("images", images_u8), ("labels", labels_u8), ("flips", flips)):
        if t is not None and (t.device.type != "cuda" or t.dtype != torch.uint8 or not t.is_contiguous()):
            raise RuntimeError(f"prep_batch: {name} must be a contiguous cuda uint8 tensor")
    n, h, w, c_img = images_u8.shape
    if c_img != 3:
        raise ValueError(f"prep_batch: images must be RGB [N,H,W,3] uint8 (got {tuple(images_u8.shape)})")
    c = _CIN[input_type]
    if labels_u8.shape != (n, h, w) or (flips is not None and flips.shape != (n,)):
        raise ValueError("prep_batch: labels must be [N,H,W] and flips [N]")
    x = torch.empty(n, c, h, w, dtype=torch.float32, device=images_u8.device)
    t = torch.empty(n, h, w, dtype=torch.float32, device=images_u8.device)
    K.call("selunet_prep_batch_mode", K.ptr(images_u8), K.ptr(labels_u8), K.ptr(flips), n, h, w, _MODE[input_type],
           K.ptr(x), K.ptr(t), K.stream_ptr())
    return x, t


class BatchLoader:
    """Global batches of a PatchSet, this rank's contiguous chunk of each, prepared on the GPU.

    shuffle: a per-epoch permutation from PCG64(seed + epoch) — identical on every rank, so the
    ranks agree on the global batch (DataLoader(shuffle=True), train.py:380). random_flip: per
    image, fliplr with p=0.5 then flipud with p=0.5 (RandomFlip, utils/data_utils.py:108-125).
    A final global batch too small to give every rank at least one image is dropped under data
    parallelism (DataParallel would run it on fewer replicas); `dropped` reports it.
    """

    def __init__(self, ds: PatchSet, batch_size: int, shuffle: bool, random_flip: bool, device, seed: int = 0,
                 max_batches: int = 0, input_type: str = "RGB"):
        self.ds, self.bs, self.shuffle, self.flip = ds, int(batch_size), shuffle, random_flip
        self.input_type = input_type
        self.device, self.seed, self.max_batches = device, seed, max_batches
        self.epoch = 0
        self.dropped = 0
        self._pool = cf.ThreadPoolExecutor(max_workers=1)
        self._copy_stream = None

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def _plan(self):
        n = len(self.ds)
        rng = np.random.Generator(np.random.PCG64(self.seed + self.epoch))
        order = rng.permutation(n) if self.shuffle else np.arange(n)
        flips = np.zeros(n, np.uint8)
        if self.flip:
            r = rng.random((n, 2))
            flips = ((r[:, 0] > 0.5) * 1 + (r[:, 1] > 0.5) * 2).astype(np.uint8)
        world, rank = parallel.world_size(), parallel.rank()
        batches = []
        for b0 in range(0, n, self.bs):
            idx = order[b0:b0 + self.bs]
            cs = -(-len(idx) // world)
            if -(-len(idx) // cs) < world:  # torch.chunk would leave a rank without images
                self.dropped += 1
                continue
            lo, hi = parallel.chunk_bounds(len(idx), rank, world)
            batches.append((len(idx), idx[lo:hi], flips[order[b0:b0 + self.bs]][lo:hi]))
        if self.max_batches:
            batches = batches[:self.max_batches]
        return batches

    def _host(self, item):
        gb, idx, fl = item
        srt = np.argsort(idx, kind="stable")  # sorted reads from a memory map, then restore the order
        inv = np.empty_like(srt)
        inv[srt] = np.arange(len(srt))
        im = torch.from_numpy(np.ascontiguousarray(self.ds.images[idx[srt]][inv])).pin_memory()
        lb = torch.from_numpy(np.ascontiguousarray(self.ds.labels[idx[srt]][inv])).pin_memory()
        return gb, im, lb, torch.from_numpy(np.ascontiguousarray(fl)).pin_memory()

    def __len__(self):
        return len(self._plan())

    def _upload(self, item, copy_stream):
        """Host batch -> device. On a GPU the copies run on `copy_stream` (an event marks their end), so
        batch i+1 crosses PCIe while step i computes instead of in front of step i+1."""
        gb, im, lb, fl = item
        if copy_stream is None:
            return gb, im.to(self.device), lb.to(self.device), fl.to(self.device), None
        with torch.cuda.stream(copy_stream):
            dev = [t.to(self.device, non_blocking=True) for t in (im, lb, fl)]
            ev = torch.cuda.Event()
            ev.record(copy_stream)
        return (gb, *dev, ev)

    def __iter__(self):
        plan = self._plan()
        if not plan:
            return
        cs = None
        if torch.device(self.device).type == "cuda":
            if self._copy_stream is None:  # (one per loader: a stream per epoch costs a creation each time)
                self._copy_stream = torch.cuda.Stream(device=self.device)
            cs = self._copy_stream
        fut = self._pool.submit(self._host, plan[0])
        pending = self._upload(fut.result(), cs)
        for i in range(len(plan)):
            if i + 1 < len(plan):
                fut = self._pool.submit(self._host, plan[i + 1])
            gb, im, lb, fl, ev = pending
            if ev is not None:  # the step's stream waits for the copies; the allocator learns the new user
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in (im, lb, fl):
                    t.record_stream(cur)
            parallel.set_global_batch(gb)
            x, t = prep_batch(im, lb, fl, self.input_type)
            yield x, t
            if i + 1 < len(plan):  # (the consumer has enqueued step i: this upload overlaps it)
                pending = self._upload(fut.result(), cs)
