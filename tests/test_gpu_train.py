"""Training-loop pieces on the GPU: batch preparation, on-device metrics, the mIoU parity run
against the reference's own training loop (tests/golden/miou_sel_256.npz, written by
tests/golden/make_golden.py from the reference model/loss/Evaluator), and the train.py CLI.

Tolerances: prep and metric counts are integer/byte work -> bit-exact. mIoU: |delta| <= 0.002
(BASELINE.json north_star) for the fp32 path, training-phase and validation alike; the bf16 path is
held to 0.01.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import selectivenet_for_semantic_segmentation_binary_amd as S
from oracle import unet_b_cpu as O
from selectivenet_for_semantic_segmentation_binary_amd import data as D
from selectivenet_for_semantic_segmentation_binary_amd.metrics import SegMetrics, logit_threshold, mean_iou
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_patches, make_patches_hard, preprocess
from tests import _golden as G
from tests.test_gpu_model import build

pytestmark = pytest.mark.gpu
DEV = "cuda"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_prep_batch_bit_exact():
    rng = np.random.Generator(np.random.PCG64(5))
    n, h, w = 5, 24, 36
    imgs = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    labs = rng.choice(np.array([0, 1, 128, 250, 254, 255], np.uint8), size=(n, h, w))
    flips = np.array([0, 1, 2, 3, 1], np.uint8)
    x, t = D.prep_batch(torch.tensor(imgs, device=DEV), torch.tensor(labs, device=DEV),
                        torch.tensor(flips, device=DEV))
    for i in range(n):
        im, lb = imgs[i], labs[i]
        if flips[i] & 1:  # RandomFlip: fliplr first, then flipud (utils/data_utils.py:113-121)
            im, lb = np.fliplr(im), np.fliplr(lb)
        if flips[i] & 2:
            im, lb = np.flipud(im), np.flipud(lb)
        xe, te = preprocess(np.ascontiguousarray(im)[None], np.ascontiguousarray(lb)[None])
        assert np.array_equal(x[i].cpu().numpy().view(np.uint32), xe[0].view(np.uint32)), i
        assert np.array_equal(t[i].cpu().numpy(), te[0]), i
    assert float(t.max()) == 1.0 and set(np.unique(t.cpu().numpy())) <= {0.0, 1.0}


@pytest.mark.parametrize("rule", ["train", "eval"])
def test_seg_metrics_bit_exact(rule):
    rng = np.random.Generator(np.random.PCG64(11))
    p = 4 * 3 * 50 + 3  # ragged tail (not a multiple of 4)
    thr = np.float32(logit_threshold(rule))
    out = rng.normal(0, 1e-6, p).astype(np.float32)
    sel = rng.normal(0, 1e-6, p).astype(np.float32)
    # values straddling the exact decision boundary, +-inf, nan, saturated
    edge = np.array([thr, np.nextafter(thr, np.float32(-1)), np.nextafter(thr, np.float32(1)), 0, -0.0, np.inf,
                     -np.inf, np.nan, 40, -40], np.float32)
    out[:len(edge)] = edge
    sel[5:5 + len(edge)] = edge
    tgt = (rng.random(p) > 0.4).astype(np.float32)
    mask = O.train_pred_mask if rule == "train" else O.eval_pred_mask
    with np.errstate(over="ignore", invalid="ignore"):
        pred, smask = mask(out), mask(sel)
    for selective in (False, True):
        m = SegMetrics(DEV, selective=selective, rule=rule)
        ot, st, tt = (torch.tensor(a, device=DEV) for a in (out, sel, tgt))
        m.add_batch(ot, tt, st)
        m.add_batch(ot, tt, st)  # accumulates
        cm = O.confusion_matrix(tgt.astype("uint8"), pred, selection=smask if selective else None)
        assert np.array_equal(m.confusion_matrix(), 2 * cm)
        selected, total = m.selected_total()
        assert total == 2 * p
        assert selected == (2 * int(smask.sum()) if selective else 2 * p)


def _loop(net, xs, ls, bs, epochs, lamb, training, metrics, cosine_min=0.0):
    loss_A = S.BCEWithLogitsLoss()
    opt = S.Adam(net.parameters(), lr=1e-3) if training else None
    # the reference's CosineAnnealingLR(T_max=epochs, eta_min=cosine_min), stepped once per epoch
    # (train.py:100-101, 246-250), as a plain torch scheduler on the package's torch-compatible Adam
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=epochs, eta_min=cosine_min) \
        if training and cosine_min > 0 else None
    losses = []
    for ep in range(epochs):
        if sched is not None and ep > 0:
            sched.step()
        for b0 in range(0, xs.shape[0], bs):
            x, lab = xs[b0:b0 + bs], ls[b0:b0 + bs]
            o, s, a = net(x)
            loss = loss_A(a, lab) + S.calc_selective_risk_image_b(o, s, target=lab, lamb=lamb)[0]
            if training:
                opt.zero_grad()
                loss.backward()
                opt.step()
            for m in metrics:
                m.add_batch(o.detach(), lab, s.detach())
            losses.append(float(loss.item()))
    return np.array(losses)


def _miou_data(d):
    """The fixture's training / validation patches (make_patches, or make_patches_hard with the
    recorded settings)."""
    size = int(d["meta_size"])
    hard = d["meta_hard"] if "meta_hard" in d.files else np.zeros(0)
    if hard.size:
        c, nz, tx, dc = (float(v) for v in hard[:4])
        tf = float(hard[4]) if hard.size > 4 else 0.39  # tumorable fraction (the selective-metric set: 0.9)
        gen = lambda n, sd: make_patches_hard(n, size, seed=sd, contrast=c, noise=nz, texture=tx,  # noqa: E731
                                              decoys=int(dc), tumorable_frac=tf)
    else:
        gen = lambda n, sd: make_patches(n, size, seed=sd)  # noqa: E731
    return (preprocess(*gen(int(d["meta_n_train"]), int(d["meta_train_seed"]))),
            preprocess(*gen(int(d["meta_n_val"]), int(d["meta_val_seed"]))))


def _has_ensemble(f):
    """A fixture is a parity gate once its reference ensemble (`val_miou_ens`) has been collected."""
    p = os.path.join(G.GOLDEN, f)
    if not os.path.exists(p):
        return False
    with np.load(p, allow_pickle=False) as d:
        return "val_miou_ens" in d.files


MIOU_FIXTURES = [f for f in ("miou_sel_256s.npz", "miou_sel_256h.npz", "miou_sel_256.npz") if _has_ensemble(f)]


@pytest.mark.parametrize("fname", MIOU_FIXTURES)
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 0.002), (torch.bfloat16, 0.01)])
def test_miou_parity_vs_reference_training(dtype, tol, fname):
    """BASELINE.json 'mIoU parity': the reference's training loop (train.py:183-241) run by
    tests/golden/make_golden.py — 16 epochs over 128 seeded synthetic 256x256 patches at batch 16,
    s_lamb=2, Adam lr 1e-3 — then eval-mode mIoU (Evaluator.get_mIoU, utils/compute_metric.py:60-65;
    prediction rule of train.py:150) over 256 validation patches; the same run through the HIP path
    must land within `tol` of the reference's training-phase and validation mIoU. Three data sets:
    miou_sel_256s.npz (make_golden.py miou256s, VERDICT r4 item 6: the selective metric the reference
    headlines, README.md:85 / eval.py:236-246 — tumour in 90 % of the patches, so the selection head must
    keep most tumour pixels and the selective val mIoU lands near 0.97, not at a degenerate value; the
    run's val coverage is held to the reference's too), miou_sel_256h.npz (make_golden.py miou256h:
    synthetic.make_patches_hard — low colour contrast, noise, a stain texture shared by both classes and
    unlabelled tumor-coloured decoys, so the reference's own validation mIoU is far from 1 and a defect
    moves it; its selection rejects the tumour) and miou_sel_256.npz (the easy set: 0.9994). Each
    fixture records the reference's own spread (runs on training inputs perturbed by 1e-7 relative,
    `val_miou_ens`; 8 and 5 members on the two discriminative sets), which must stay within 1.5x of the fp32
    bar; the printed line also gives ours as a z-score against that ensemble."""
    d = G.load(fname)
    bs, ep, lamb = int(d["meta_bs"]), int(d["meta_epochs"]), int(d["meta_lamb"])
    (xtr, ltr), (xva, lva) = _miou_data(d)
    net = build(True, int(d["meta_seed"]), dtype)
    tr = SegMetrics(DEV, selective=True, rule="train")
    cmin = float(d["meta_cosine_min"]) if "meta_cosine_min" in d.files else 0.0
    losses = _loop(net, torch.tensor(xtr, device=DEV), torch.tensor(ltr, device=DEV), bs, ep, lamb, True, [tr], cmin)
    ref_losses = d["train_losses"]
    print(f"train loss {losses[0]:.5f}->{losses[-1]:.5f} (reference {ref_losses[0]:.5f}->{ref_losses[-1]:.5f})")
    assert abs(losses[0] - ref_losses[0]) < (1e-4 if dtype == torch.float32 else 2e-2) * abs(ref_losses[0])
    assert np.abs(losses - ref_losses).max() < 0.05 * max(1.0, np.abs(ref_losses).max())
    m_tr, m_tr_ref = mean_iou(tr.confusion_matrix()), mean_iou(d["train_cm"])
    net.eval()
    vs, vp = SegMetrics(DEV, selective=True, rule="train"), SegMetrics(DEV, selective=False, rule="train")
    with torch.no_grad():
        _loop(net, torch.tensor(xva, device=DEV), torch.tensor(lva, device=DEV), bs, 1, lamb, False, [vs, vp])
    m_sel, m_all = mean_iou(vs.confusion_matrix()), mean_iou(vp.confusion_matrix())
    spread = {k: float(np.abs(d[k + "_ens"] - float(d[k])).max()) for k in ("val_miou", "val_miou_selective")
              if k + "_ens" in d.files}
    # where ours sits in the reference's own distribution (the unperturbed run and its members)
    zs = {}
    for k, got in (("val_miou", m_all), ("val_miou_selective", m_sel)):
        if k + "_ens" in d.files:
            ens = np.concatenate([[float(d[k])], d[k + "_ens"]])
            zs[k] = (got - ens.mean()) / max(ens.std(ddof=1), 1e-9)
    line = (f"mIoU {fname} [{dtype}]: train {m_tr:.5f} (reference {m_tr_ref:.5f}), val {m_all:.5f} (reference "
            f"{float(d['val_miou']):.5f}), val selective {m_sel:.5f} (reference {float(d['val_miou_selective']):.5f}); "
            f"reference spread {spread}; z vs the reference ensemble {({k: round(float(v), 2) for k, v in zs.items()})}; "
            f"tol {tol}")
    print(line)
    G.SUMMARY.append(line)
    # the set discriminates at the scale of the fp32 bar: the reference's own members (1e-7 input perturbations,
    # 16 epochs of chaotic training) scatter by at most 1.5x of it around its unperturbed run
    assert spread and max(spread.values()) < 0.003, ("the reference's own spread must stay near the bar", spread)
    if "ens_members" in d.files:  # collected by make_golden.py miou256x_collect: >= 5 reference members
        assert d["val_miou_ens"].size >= 5, d["val_miou_ens"].size  # (miou_sel_256s: 8, miou_sel_256h: 5)
    assert abs(m_tr - m_tr_ref) <= tol
    for got, key in ((m_all, "val_miou"), (m_sel, "val_miou_selective")):
        # against the reference's distribution where it was sampled: one 16-epoch run is one draw of a chaotic
        # process (the reference's own members sit up to 0.0021 from its unperturbed run on miou_sel_256s, so
        # a single-run bar would fail the reference itself); the bar is on the ensemble mean. (No z-score bar:
        # 1e-7 input perturbations understate what a different fp32 summation order does to 16 epochs — our own
        # runs moved by 0.0015 on miou_sel_256h when one kernel's BN-sum order changed, against a member std of
        # 0.0004 there; the z-score is printed)
        if key + "_ens" in d.files:
            ens = np.concatenate([[float(d[key])], d[key + "_ens"]])
            assert abs(got - ens.mean()) <= tol, (key, got, float(ens.mean()))
        else:
            assert abs(got - float(d[key])) <= tol, (key, got, float(d[key]))
    if fname == "miou_sel_256s.npz":
        # the selective metric is not degenerate here, and the selection keeps as many pixels as the reference's
        assert 0.85 <= float(d["val_miou_selective"]) <= 0.99, float(d["val_miou_selective"])
        sel_ours, total = vs.selected_total()
        cov, cov_ref = sel_ours / total, float(d["val_selected"]) / total
        cov_spread = float(np.abs(d["val_selected_ens"] - float(d["val_selected"])).max()) / total
        print(f"val coverage {cov:.5f} (reference {cov_ref:.5f}, spread {cov_spread:.5f})")
        assert abs(cov - cov_ref) <= max(3 * cov_spread, 0.005), (cov, cov_ref, cov_spread)


def _cli(tmp, *extra):
    cmd = [sys.executable, "-m", "selectivenet_for_semantic_segmentation_binary_amd.train", "--data_dir",
           "synthetic:40", "--patch_size", "64", "--model_arch", "UNet_B", "--loss", "BCElogit", "--selective", "1",
           "--batch_size", "8", "--model_dir", str(tmp), "--steps_per_epoch", "3", "--val_steps", "1", *extra]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_cli_epochs_checkpoints_resume(tmp_path):
    out = _cli(tmp_path, "--n_epoch", "2", "--lr_sche", "StepLR", "--patience", "1")
    assert "train_loss" in out and "train_rejection" in out and "valid_rejection" in out
    ck = tmp_path / "1-fold" / "checkpoint"
    assert sorted(os.listdir(ck)) == ["model_epoch1.pth", "model_epoch2.pth"]
    sd = torch.load(ck / "model_epoch2.pth", map_location="cpu", weights_only=True)
    assert list(sd["net"].keys()) == S.state_dict_keys("RGB", True)
    assert int(sd["net"]["encoder_layer_1_1.1.num_batches_tracked"]) == 6
    assert len(sd["optim"]["state"]) == len(sd["net"]) - 3 * 14  # params only (no BN buffers)
    hist = json.load(open(tmp_path / "1-fold" / "log" / "history.json"))
    assert [h["epoch"] for h in hist] == [1, 2]
    assert all(sum(map(sum, h["train_cm"])) > 0 for h in hist)
    # resume: the newest checkpoint's weights, epoch numbering continues (train.py:113-127)
    out2 = _cli(tmp_path, "--n_epoch", "1")
    assert "Load weights from" in out2 and "epoch 3 / 3" in out2
    assert sorted(os.listdir(ck))[-1] == "model_epoch3.pth"


def test_eval_cli_matches_oracle_metrics(tmp_path):
    """eval.py mirror on a checkpoint written by the train CLI: the device Evaluator's confusion
    matrix equals the CPU oracle's eval-mode forward + the reference's fp32 sigmoid rule
    (eval.py:175,179,233) + Evaluator (utils/compute_metric.py:10-26), up to pixels whose logit
    lies within fp32 rounding of the cut (<= 1e-3 of the pixels)."""
    _cli(tmp_path, "--n_epoch", "1")
    ck = tmp_path / "1-fold" / "checkpoint"
    out = tmp_path / "eval_out"
    cmd = [sys.executable, "-m", "selectivenet_for_semantic_segmentation_binary_amd.eval", "--data_dir", "synthetic:8",
           "--patch_size", "64", "--test_fold", "2", "--model_dir", str(ck), "--model_arch", "UNet_B",
           "--selective", "1", "--select_eval", "1", "--batch_size", "4", "--save_dir", str(out)]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "mIoU:" in r.stdout and "rejection ratio:" in r.stdout
    res = json.load(open(out / "performance.json"))

    sd = torch.load(ck / "model_epoch1.pth", map_location="cpu", weights_only=True)["net"]
    params, buffers = O.make_state(0, "RGB", True)
    with torch.no_grad():
        for k in params:
            params[k].copy_(sd[k])
        for k in buffers:
            buffers[k].copy_(sd[k])
    from selectivenet_for_semantic_segmentation_binary_amd.data import load_test_set_for_tests
    imgs, labs = load_test_set_for_tests("synthetic:8", 64, 2)
    x, lab = preprocess(imgs, labs)
    with torch.no_grad():
        o, s, _ = O.forward(params, buffers, torch.tensor(x), True, training=False)
    pred = O.eval_pred_mask(o.numpy())
    sel = O.eval_pred_mask(s.numpy())
    cm = O.confusion_matrix(lab.astype("uint8"), pred, selection=sel)
    got = np.array(res["confusion_matrix"])
    assert np.abs(got - cm).sum() <= 1e-3 * lab.size, (got, cm)
    assert abs(res["rejection_ratio"] - (1 - sel.mean())) <= 1e-3


def test_train_cli_ce_unet(tmp_path):
    """--model_arch UNet --loss CE (the reference's defaults, train.py:42,54): CE UNet, CrossEntropyLoss
    aux + calc_selective_risk_image, argmax masks; checkpoint in the reference's UNet layout."""
    out = _cli(tmp_path, "--model_arch", "UNet", "--loss", "CE", "--n_epoch", "1")
    assert "train_loss" in out and "train_rejection" in out
    sd = torch.load(tmp_path / "1-fold" / "checkpoint" / "model_epoch1.pth", map_location="cpu", weights_only=True)
    assert list(sd["net"].keys()) == S.state_dict_keys("RGB", True, n_cls=2)
    assert tuple(sd["net"]["conv_select.weight"].shape) == (2, 64, 1, 1)
    hist = json.load(open(tmp_path / "1-fold" / "log" / "history.json"))
    assert np.isfinite(hist[0]["train_loss"]) and 0 < sum(map(sum, hist[0]["train_cm"])) <= 3 * 8 * 64 * 64  # selected px
