"""Training CLI mirroring the reference's train.py on the MI355X path.

    python -m selectivenet_for_semantic_segmentation_binary_amd.train --fold 1 --data_dir /data \\
        --model_dir /model --model_arch UNet_B --selective 1 --loss BCElogit \\
        --local_rank 0 1 2 3 4 5 6 7 --n_epoch 200 --batch_size 128          (train.sh)

Same flags, defaults and argument meanings as train.py:12-55 (including argparse's `type=bool`
quirk: any non-empty value of --selective / --log_img is True), same epoch loop
(train.py:161-345), same printed lines, same checkpoint layout `{model_dir}/{fold}-fold/checkpoint/
model_epoch{E}.pth` = {'net', 'optim'} (utils/net_utils.py:5-9) and the same resume rule (newest
checkpoint by the digits of its name, network weights only, train.py:113-127).

What differs, by design:
  * `--local_rank 0 1 ... 7` spawns one process per listed GPU id (RCCL all-reduce over xGMI,
    `parallel`) instead of wrapping the model in torch.nn.DataParallel; a single id runs on that
    GPU (the reference's single-GPU branch crashes on `cuda:[0]`).
  * The forward/backward/loss/Adam run in libselunet.so (HIP, gfx950); `--compute_dtype bf16`
    selects the bf16 MFMA path (default fp32 = the reference's arithmetic).
  * Per-step metrics (thresholds, rejection counts, confusion matrix) and loss sums stay on the
    GPU (`metrics.SegMetrics`) and are read once per epoch, instead of copying every batch's
    outputs to the host.
  * Data: `--data_dir synthetic[:N]` uses the seeded synthetic patches; any other
    directory is read through the reference's split files ({k}-fold_{,non_}tumorable_data.npy) and
    decoded once into uint8 caches (`data.decode_patch_list`); normalisation and flips run on the
    GPU. input_type 'RGB', 'GH' or 'H_RGB'; model_arch 'UNet_B' with loss 'BCElogit', or the CE `UNet`
    (model_arch 'UNet', loss 'CE', n_cls 2: CrossEntropyLoss aux + calc_selective_risk_image, argmax
    masks as train.py:207-219).
  * TensorBoard scalars are written when torch.utils.tensorboard is importable, otherwise as JSON
    lines in `{log_dir}/{train,valid}/scalars.jsonl`.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np


def parse_arguments(argv=None):
    """train.py:12-55, plus MI355X-path options (after the reference's)."""
    parser = argparse.ArgumentParser()
    parser.add_argument('--data_dir', type=str, help='WSI data directory', default='/data')
    parser.add_argument('--fold', type=int, default=1, help='which fold in 5-fold cv')
    parser.add_argument('--input_type', type=str, default='RGB')
    parser.add_argument('--patch_mag', type=int, default=200)
    parser.add_argument('--patch_size', type=int, default=256)
    parser.add_argument('--n_cls', type=int, default=2)
    parser.add_argument('--model_dir', type=str, help='directory where logs and models would be saved',
                        default='/model')
    parser.add_argument('--model_arch', type=str, default='UNet', choices=['UNet', 'UNet_B'])
    parser.add_argument('--selective', type=bool, default=False, help='Is the network based on SelectiveNet?')
    parser.add_argument('--s_lamb', type=int, default=2, help='degree to follow target coverage')
    parser.add_argument('--output_dim', type=str, default='NHW', choices=['NCHW', 'NHW'])
    parser.add_argument('--output_scale', type=str, default='sigmoid', choices=['None', 'clip', 'sigmoid', 'minmax'])
    parser.add_argument('--optim', type=str, default='Adam', choices=['Adam', 'SGD'])
    parser.add_argument('--momentum', type=float, default=0, choices=[0.9])
    parser.add_argument('--w_decay', type=float, default=0, choices=[5e-4])
    parser.add_argument('--lr', type=float, default=1e-3)
    parser.add_argument('--lr_sche', type=str, default=None, choices=['StepLR', 'ReduceLR', 'CosineAnnealingLR'])
    parser.add_argument('--patience', type=int, default=10)
    parser.add_argument('--factor', type=float, default=0.5)
    parser.add_argument('--lr_min', type=float, default=1e-5)
    parser.add_argument('--loss', type=str, default='CE', choices=['BCElogit', 'CE'])
    parser.add_argument('--batch_size', type=int, default=16)
    parser.add_argument('--n_epoch', type=int, default=100)
    parser.add_argument('--local_rank', type=int, nargs='+', default=[0], help='local rank')
    parser.add_argument('--log_img', type=bool, default=False)
    # ---- MI355X path options
    parser.add_argument('--compute_dtype', type=str, default='fp32', choices=['fp32', 'bf16'],
                        help='activation/MFMA operand type (fp32 = reference arithmetic)')
    parser.add_argument('--seed', type=int, default=0, help='init / shuffle / flip seed')
    parser.add_argument('--steps_per_epoch', type=int, default=0, help='cap on training batches per epoch (0 = all)')
    parser.add_argument('--val_steps', type=int, default=0, help='cap on validation batches per epoch (0 = all)')
    parser.add_argument('--quiet', action='store_true')
    return parser.parse_args(argv)


# ----------------------------------------------------------------------------- process launch
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(argv, gpu_ids, command=None):
    """One child process per listed GPU id (replaces torch.nn.DataParallel(device_ids=rank),
    train.py:131-134). The parent never touches the GPU; it waits and returns the exit code of the
    first child that failed on its own (the siblings it then terminates exit with -SIGTERM, which is
    not reported).
    command: the child command line (default: this module with `argv`)."""
    port = str(_free_port())
    procs = []
    cmd = command or [sys.executable, "-m", __spec__.name if __spec__ else __name__, *argv]
    for r, gid in enumerate(gpu_ids):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(len(gpu_ids)),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, SELUNET_GPU_ID=str(gid))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    terminated = set()  # children this function stopped: their -SIGTERM is not the job's failure
    try:
        # poll every child: the first non-zero exit (of any rank, not just the next one in order)
        # ends the job at once instead of leaving the others blocked in a collective until the
        # process-group timeout
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and p.pid not in terminated and rc == 0:
                    rc = code if code > 0 else 128 - code
                if code != 0:
                    for q in live:
                        terminated.add(q.pid)
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


# ----------------------------------------------------------------------------- logging
class _Scalars:
    def __init__(self, log_dir, enabled):
        self.enabled = enabled
        self.tb = None
        if not enabled:
            return
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.tb = SummaryWriter(log_dir=log_dir)
        except Exception:  # tensorboard is not installed in this image
            os.makedirs(log_dir, exist_ok=True)
            self.path = os.path.join(log_dir, "scalars.jsonl")

    def add_scalar(self, tag, value, step):
        if not self.enabled:
            return
        if self.tb is not None:
            self.tb.add_scalar(tag, value, step)
        else:
            with open(self.path, "a") as fh:
                fh.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")

    def close(self):
        if self.tb is not None:
            self.tb.close()


# ----------------------------------------------------------------------------- data
def load_data(args, seed):
    from . import data as D

    if args.data_dir.startswith("synthetic"):
        n = int(args.data_dir.split(":")[1]) if ":" in args.data_dir else 512
        full = D.synthetic_patchset(n, args.patch_size, seed=1000 + seed)
        # 5 folds by index; the test fold is held out, 20% of the rest validates (train.py:369-374)
        fold = np.arange(n) % 5 + 1
        rest = np.nonzero(fold != args.fold)[0]
        rs = np.random.RandomState(42)
        vidx = np.sort(rs.choice(len(rest), size=int(len(rest) * 0.2), replace=False))
        tidx = np.setdiff1d(np.arange(len(rest)), vidx)
        pick = lambda ix: D.PatchSet(full.images[rest[ix]], full.labels[rest[ix]])  # noqa: E731
        return pick(tidx), pick(vidx)
    train_list, valid_list = D.construct_train_valid(args.data_dir, test_fold=args.fold)
    return (D.decode_patch_list(args.data_dir, train_list, args.patch_mag, args.patch_size),
            D.decode_patch_list(args.data_dir, valid_list, args.patch_mag, args.patch_size))


# ----------------------------------------------------------------------------- training
def train(args, ckpt_dir, log_dir):
    import torch

    import selectivenet_for_semantic_segmentation_binary_amd as S
    from . import data as D
    from . import net_utils, parallel
    from .metrics import SegMetrics, pixel_accuracy

    ce = args.model_arch == 'UNet'
    if (ce and args.loss != 'CE') or (not ce and args.loss != 'BCElogit'):
        raise NotImplementedError("the MI355X path pairs model_arch 'UNet_B' with loss 'BCElogit' and 'UNet' "
                                  "with 'CE' (train.py:71-86 allows the mixed pairs; they are not implemented)")
    if ce and args.n_cls != 2:
        raise NotImplementedError("the CE UNet's on-device metrics are binary: n_cls 2 (train.py:23 default)")
    if args.input_type not in ('RGB', 'GH', 'H_RGB'):
        raise ValueError(f"input_type {args.input_type!r}: 'RGB', 'GH' or 'H_RGB' (utils/data_utils.py:223-226)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = int(os.environ.get("SELUNET_GPU_ID", args.local_rank[0]))
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    rank = 0
    if world > 1:
        rank, world = parallel.init_data_parallel("nccl")
    log = (lambda *a: print(*a, flush=True)) if rank == 0 and not args.quiet else (lambda *a: None)  # noqa: E731

    torch.manual_seed(args.seed)
    dt = torch.bfloat16 if args.compute_dtype == 'bf16' else torch.float32
    if ce:
        net = S.UNet(args.input_type, args.n_cls, selective=args.selective, compute_dtype=dt)
        loss_A = S.CrossEntropyLoss()
        loss_S = S.calc_selective_risk_image if args.selective else None
    else:
        net = S.UNet_B(args.input_type, selective=args.selective, compute_dtype=dt)
        loss_A = S.BCEWithLogitsLoss()
        loss_S = S.calc_selective_risk_image_b if args.selective else None

    start_epoch = 0
    if os.path.exists(ckpt_dir) and os.listdir(ckpt_dir):  # train.py:113-127 (network weights only)
        names = sorted(os.listdir(ckpt_dir), key=lambda f: int(''.join(filter(str.isdigit, f))))
        net_utils.net_test_load(os.path.join(ckpt_dir, names[-1]), net)
        start_epoch = int(names[-1].split('epoch')[1].split('.pth')[0])
        log('Load weights from', os.path.join(ckpt_dir, names[-1]))
    net = net.to(device)
    parallel.broadcast_params(net)

    if args.optim == 'Adam':
        optim = S.Adam(net.parameters(), lr=args.lr, weight_decay=args.w_decay)
    else:
        optim = torch.optim.SGD(net.parameters(), lr=args.lr, momentum=args.momentum, weight_decay=args.w_decay)
    scheduler = None
    if args.lr_sche == 'StepLR':
        scheduler = torch.optim.lr_scheduler.StepLR(optim, step_size=args.patience, gamma=args.factor)
    elif args.lr_sche == 'ReduceLR':
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optim, mode='min', patience=args.patience,
                                                               factor=args.factor)
    elif args.lr_sche == 'CosineAnnealingLR':
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optim, T_max=args.patience, eta_min=args.lr_min)

    ds_train, ds_val = load_data(args, args.seed)
    loader_train = D.BatchLoader(ds_train, args.batch_size, shuffle=True, random_flip=True, device=device,
                                 seed=args.seed, max_batches=args.steps_per_epoch, input_type=args.input_type)
    loader_val = D.BatchLoader(ds_val, args.batch_size, shuffle=False, random_flip=False, device=device,
                               seed=args.seed, max_batches=args.val_steps, input_type=args.input_type)
    log(f'# of gpu: {world}, gpu id: {args.local_rank}\n')

    writer_train = _Scalars(os.path.join(log_dir, 'train'), rank == 0)
    writer_val = _Scalars(os.path.join(log_dir, 'valid'), rank == 0)
    rule = "argmax" if ce else "train"
    ev_train = SegMetrics(device, selective=bool(args.selective), rule=rule, output_scale=args.output_scale)
    ev_val = SegMetrics(device, selective=bool(args.selective), rule=rule, output_scale=args.output_scale)

    def binary(t):  # CE logits (N, 2, H, W) -> the fp32 difference the argmax rule thresholds at 0
        return (t[:, 1] - t[:, 0]).contiguous() if ce else t
    history = []

    def run_epoch(loader, training, ev):
        sums = torch.zeros(3, dtype=torch.float64, device=device)  # loss, aux loss, selection loss
        steps = 0
        for x, target in loader:
            tgt = target.long() if ce else target  # train.py:189-191 (int64 labels for CE)
            if args.selective:
                output, selection, aux = net(x)
                aux_loss = loss_A(aux, tgt)
                select_loss, coverage = loss_S(output, selection, target=tgt, lamb=args.s_lamb)
                loss = aux_loss + select_loss
                sums[1] += aux_loss.detach()
                sums[2] += select_loss.detach()
            else:
                output, selection = net(x), None
                loss = loss_A(output, tgt)
            if training:
                optim.zero_grad()
                loss.backward()
                optim.step()
            sums[0] += loss.detach()
            ev.add_batch(binary(output.detach()), target, None if selection is None else binary(selection.detach()))
            steps += 1
        return sums, steps

    for epoch in range(start_epoch + 1, start_epoch + args.n_epoch + 1):
        current_lr = optim.param_groups[-1]['lr']
        writer_train.add_scalar('lr', current_lr, epoch)
        log(f'epoch {epoch} / {start_epoch + args.n_epoch}, learning rate {current_lr}')
        t0 = time.perf_counter()
        net.train()
        loader_train.set_epoch(epoch)
        ev_train.reset()
        tr_sums, tr_steps = run_epoch(loader_train, True, ev_train)
        torch.cuda.synchronize()
        t_train = time.perf_counter() - t0
        tr = (tr_sums / max(tr_steps, 1)).cpu().numpy()
        tr_cm = ev_train.confusion_matrix()
        tr_sel, tr_total = ev_train.selected_total()
        tr_acc = pixel_accuracy(tr_cm)
        if scheduler is not None:
            scheduler.step(tr[0]) if args.lr_sche == 'ReduceLR' else scheduler.step()

        with torch.no_grad():
            net.eval()
            ev_val.reset()
            va_sums, va_steps = run_epoch(loader_val, False, ev_val)
        va = (va_sums / max(va_steps, 1)).cpu().numpy()
        va_cm = ev_val.confusion_matrix()
        va_sel, va_total = ev_val.selected_total()
        va_acc = pixel_accuracy(va_cm)

        writer_train.add_scalar('loss', tr[0], epoch)
        writer_train.add_scalar('accuracy', tr_acc, epoch)
        writer_val.add_scalar('loss', va[0], epoch)
        writer_val.add_scalar('accuracy', va_acc, epoch)
        tr_rej = (tr_total - tr_sel) / max(tr_total, 1)
        va_rej = (va_total - va_sel) / max(va_total, 1)
        if args.selective:
            for w, v, rej in ((writer_train, tr, tr_rej), (writer_val, va, va_rej)):
                w.add_scalar('aux loss', v[1], epoch)
                w.add_scalar('selection loss', v[2], epoch)
                w.add_scalar('rejection ratio', rej, epoch)
        log('train_loss %.05f train_acc %.04f | valid_loss %.05f valid_acc %.04f' % (tr[0], tr_acc, va[0], va_acc))
        if args.selective:
            log('train_aux_loss %.05f | train_select_loss %.05f | train_rejection %.03f' % (tr[1], tr[2], tr_rej))
            log('valid_aux_loss %.05f | valid_select_loss %.05f | valid_rejection %.03f' % (va[1], va[2], va_rej))
        imgs = tr_steps * args.batch_size
        log(f'train throughput {imgs / t_train:.1f} images/s over {tr_steps} steps ({world} GPU)')
        history.append({"epoch": epoch, "train_loss": float(tr[0]), "train_acc": float(tr_acc),
                        "valid_loss": float(va[0]), "valid_acc": float(va_acc), "train_cm": tr_cm.tolist(),
                        "valid_cm": va_cm.tolist(), "train_rejection": tr_rej, "valid_rejection": va_rej,
                        "train_images_per_s": imgs / t_train})
        if rank == 0:  # DataParallel replica 0's buffers are the ones the reference saves
            net_utils.net_save(ckpt_dir=ckpt_dir, net=net, optim=optim, epoch=epoch)
    writer_train.close()
    writer_val.close()
    if rank == 0:
        os.makedirs(log_dir, exist_ok=True)
        with open(os.path.join(log_dir, "history.json"), "w") as fh:
            json.dump(history, fh, indent=1)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    return history


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_arguments(argv)
    if len(args.local_rank) > 1 and "RANK" not in os.environ:
        return spawn(argv, args.local_rank)
    if not args.quiet and os.environ.get("RANK", "0") == "0":
        print('')
        print('args={}\n'.format(args))
    ckpt_dir = f'{args.model_dir}/{args.fold}-fold/checkpoint'
    log_dir = f'{args.model_dir}/{args.fold}-fold/log'
    train(args, ckpt_dir, log_dir)
    return 0


if __name__ == '__main__':
    sys.exit(main())
