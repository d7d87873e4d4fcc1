"""Evaluation CLI mirroring the reference's eval.py on the MI355X path (forward-only).

    python -m selectivenet_for_semantic_segmentation_binary_amd.eval --data_dir /data --test_fold 1 \\
        --model_dir /model/1-fold/checkpoint --model_arch UNet_B --selective 1 --select_eval 1

Same flags and defaults as eval.py:17-58 (argparse `type=bool` quirk included), same model loading
(every *.pth in --model_dir, sorted, `module.` prefixes stripped, eval.py:116-154), same
prediction rule — fp32 numpy sigmoid then `> --cut_off` (eval.py:171,175,229-231), selection
`> --s_cut_off` when --select_eval (eval.py:236-246) — and the same Evaluator report
(eval.py:258-279). The forward runs in eval mode with the running BatchNorm statistics on the GPU;
masks and the confusion matrix are computed on the device (`metrics.SegMetrics`, thresholds exact
by construction) and read once at the end.

Ensembles (several checkpoints, selective off, eval.py:185-199) average the per-model outputs on
the GPU in the reference's order; with --ens_scale sigmoid the GPU's exp differs from numpy's by
an ulp on some pixels (parity unpinned for that mode); None / clip / minmax are exact.
A single process evaluates on the first id of --local_rank (the reference's DataParallel split
of an eval batch changes nothing in eval mode).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def parse_arguments(argv=None):
    """eval.py:17-58."""
    parser = argparse.ArgumentParser()
    parser.add_argument('--data_dir', type=str, default='./data')
    parser.add_argument('--test_fold', type=int, default=1, help='which fold in 5-fold cv')
    parser.add_argument('--input_type', type=str, default='RGB')
    parser.add_argument('--patch_mag', type=int, default=200)
    parser.add_argument('--patch_size', type=int, default=256)
    parser.add_argument('--n_cls', type=int, default=2)
    parser.add_argument('--batch_size', type=int, default=16)
    parser.add_argument('--num_workers', type=int, default=16, help='Dataloader num_workers')
    parser.add_argument('--model_dir', type=str, default='*/model', help='network ckpt (.pth) directory')
    parser.add_argument('--model_arch', type=str, nargs='+', default=['UNet_B'], choices=['UNet_B'])
    parser.add_argument('--selective', type=bool, default=False, help='Is the network based on SelectiveNet?')
    parser.add_argument('--select_eval', type=bool, default=False, help='calculate metrics with/without selection')
    parser.add_argument('--output_dim', type=str, default='NHW', choices=['NCHW', 'NHW'])
    parser.add_argument('--single_scale', type=str, default='sigmoid', choices=['None', 'clip', 'sigmoid', 'minmax'])
    parser.add_argument('--ens_scale', type=str, default='None', choices=['None', 'clip', 'sigmoid', 'minmax'])
    parser.add_argument('--cut_off', type=float, default=0.5, help='prob > cut_off -> pred: 1')
    parser.add_argument('--s_cut_off', type=float, default=0.5, help='selection > cut_off -> select: 1')
    parser.add_argument('--local_rank', type=int, nargs='+', default=[0], help='local gpu ids')
    parser.add_argument('--info_print', type=bool, default=False)
    parser.add_argument('--save_dir', type=str, default='./output', help='saving results')
    # ---- MI355X path options
    parser.add_argument('--compute_dtype', type=str, default='fp32', choices=['fp32', 'bf16'])
    return parser.parse_args(argv)


def load_test_set(args):
    from . import data as D

    if args.data_dir.startswith("synthetic"):
        return D.PatchSet(*D.load_test_set_for_tests(args.data_dir, args.patch_size, args.test_fold))
    test_list = D.construct_test(args.data_dir, test_fold=args.test_fold)
    return D.decode_patch_list(args.data_dir, test_list, args.patch_mag, args.patch_size)


def evaluate(args):
    import torch

    import selectivenet_for_semantic_segmentation_binary_amd as S
    from . import data as D
    from . import metrics as MT
    from . import net_utils

    if args.input_type not in ('RGB', 'GH', 'H_RGB'):
        raise ValueError(f"input_type {args.input_type!r}: 'RGB', 'GH' or 'H_RGB' (utils/data_utils.py:223-226)")
    device = torch.device("cuda", args.local_rank[0])
    torch.cuda.set_device(device)
    dt = torch.bfloat16 if args.compute_dtype == 'bf16' else torch.float32
    model_list = sorted(c for c in os.listdir(args.model_dir) if 'pth' in c)
    if not model_list:
        raise FileNotFoundError(f"no .pth checkpoints in {args.model_dir}")
    arch = args.model_arch * len(model_list) if len(args.model_arch) == 1 else args.model_arch
    nets = []
    for name, a in zip(model_list, arch):
        if args.info_print:
            print(f'    {os.path.join(args.model_dir, name)} - {a} / SelectiveNet: {args.selective}')
        net = S.UNet_B(args.input_type, selective=args.selective, compute_dtype=dt)
        net_utils.net_test_load(os.path.join(args.model_dir, name), net)
        nets.append(net.to(device).train(False))
    if len(nets) > 1 and args.selective:
        raise NotImplementedError("ensembles of selective networks are not supported (eval.py:185, '선택 불가')")

    ds = load_test_set(args)
    loader = D.BatchLoader(ds, args.batch_size, shuffle=False, random_flip=False, device=device,
                           input_type=args.input_type)
    ev = MT.SegMetrics(device, selective=bool(args.select_eval), rule="eval", cut_off=args.cut_off,
                       s_cut_off=args.s_cut_off, output_scale=args.single_scale)
    print("Model Prediction...")
    with torch.no_grad():
        for x, target in loader:
            selection = None
            if len(nets) == 1:
                if args.selective:
                    output, selection, _ = nets[0](x)
                else:
                    output = nets[0](x)
            else:
                acc = None
                for net in nets:  # eval.py:185-199: mean of the scaled outputs, in model order
                    o = net(x)
                    if args.ens_scale == 'clip':
                        o = o.clamp(0, 1)
                    elif args.ens_scale == 'minmax':
                        o = (o - o.min()) / (o.max() - o.min())
                    elif args.ens_scale == 'sigmoid':
                        o = 1 / (1 + torch.exp(-o))
                    acc = o.clone() if acc is None else acc.add_(o)
                output = acc.div_(float(len(nets)))
            if args.select_eval and selection is None:
                raise ValueError("--select_eval needs a selective network (--selective 1)")
            ev.add_batch(output.contiguous(), target, None if selection is None else selection.contiguous())
    cm = ev.confusion_matrix()
    selected, total = ev.selected_total()
    prec, rec = MT.precision(cm), MT.recall(cm)
    with np.errstate(invalid="ignore", divide="ignore"):
        f1 = 2 * (prec * rec) / (prec + rec)
        acc_class = np.nanmean(np.diag(cm) / cm.sum(axis=1))
        iou_class = np.diag(cm) / (cm.sum(1) + cm.sum(0) - np.diag(cm))
    res = {"confusion_matrix": cm.tolist(), "Acc": float(MT.pixel_accuracy(cm)), "Acc_class": float(acc_class),
           "Prec": prec.tolist(), "Recall": rec.tolist(), "F1_Score": f1.tolist(), "mIoU": float(MT.mean_iou(cm)),
           "IoU_class": iou_class.tolist()}
    print(cm)
    if args.select_eval:
        res["rejection_ratio"] = (total - selected) / max(total, 1)
        print(f'    rejection ratio: {round(res["rejection_ratio"], 3)}')
    print(f'    Acc:{res["Acc"]}')
    print(f'    Acc_class:{res["Acc_class"]}')
    print(f'    Prec:{prec}, Recall:{rec}, F1_Score:{f1}')
    print(f'    mIoU:{res["mIoU"]}')
    print(f'    IoU_class:{iou_class}')
    os.makedirs(args.save_dir, exist_ok=True)
    with open(os.path.join(args.save_dir, "performance.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    return res


def main(argv=None):
    args = parse_arguments(sys.argv[1:] if argv is None else argv)
    print('')
    print('args={}\n'.format(args))
    evaluate(args)
    return 0


if __name__ == '__main__':
    sys.exit(main())
