"""The data path's host side against the oracle restatement (oracle/data_cpu.py) of the reference's
PatchDataset / Normalization / RandomFlip / ToTensor / fold splits (utils/data_utils.py:49-236):
split lists identical, PIL-decoded uint8 patches identical, the preprocessing rules on
hand-computed values. Integer/byte work: bit-exact. (GPU side: tests/test_gpu_data.py.)"""
import numpy as np

from oracle import data_cpu as OD
from selectivenet_for_semantic_segmentation_binary_amd import data as D
from tests._patchdir import make_patch_dir


def test_fold_splits_match_reference_rule(tmp_path):
    root = make_patch_dir(str(tmp_path), per_fold=10)
    for fold in (1, 3, 5):
        tr, va = D.construct_train_valid(root, test_fold=fold)
        otr, ova = OD.construct_train_valid(root, test_fold=fold)
        assert np.array_equal(tr, otr) and np.array_equal(va, ova)
        assert np.array_equal(D.construct_test(root, test_fold=fold), OD.construct_test(root, test_fold=fold))


def test_decode_matches_reference_getitem(tmp_path):
    root = make_patch_dir(str(tmp_path), per_fold=4)
    tr, _ = D.construct_train_valid(root, test_fold=5)
    for cache in (False, True, True):  # second cached call memory-maps the .npy cache
        ps = D.decode_patch_list(root, tr, patch_mag=200, patch_size=32, cache=cache)
        for i, (a, b) in enumerate(tr):
            inp, lab, pid = OD.read_patch(root, str(a), str(b), 200, 32)
            assert np.array_equal((np.asarray(ps.images[i]) / 255.0).astype(np.float32), inp)
            assert np.array_equal((np.asarray(ps.labels[i]) / 255.0).astype(np.uint8), lab)
            assert ps.ids[i] == pid
        assert (np.asarray(ps.labels) == 254).any()  # the truncation case is exercised


def test_transform_rules_on_known_values():
    inp = np.array([[[0, 127, 255]]], np.uint8) / 255.0
    lab = np.array([[254]], np.uint8) / 255.0
    x, t = OD.transform(inp.astype(np.float32), lab.astype(np.uint8), train=False)
    assert x.dtype == np.float32 and x.shape == (3, 1, 1)
    assert x[0, 0, 0] == -1.0 and x[2, 0, 0] == 1.0
    assert x[1, 0, 0] == np.float32((np.float32(127 / 255.0) - 0.5) / 0.5)
    assert t[0, 0] == 0.0  # 254/255 truncates to 0; only 255 is tumor
    im = np.arange(2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3)
    lb = np.arange(6, dtype=np.uint8).reshape(2, 3)
    x, t = OD.transform(im, lb, flips=3)  # fliplr then flipud (utils/data_utils.py:113-121)
    assert np.array_equal(t, lb[::-1, ::-1].astype(np.float32))
    assert np.array_equal(x, ((im[::-1, ::-1] - 0.5) / 0.5).transpose(2, 0, 1))


# ----------------------------------------------------------------------------- reference fixture
def _fixture_dir(tmp_path):
    """The patch directory data_rgb_n30_32.npz was recorded on (tests/golden/make_golden.py data),
    regenerated, with every file's bytes checked against the recorded SHA-1."""
    import hashlib
    import os

    from tests import _golden as G
    d = G.load("data_rgb_n30_32.npz")
    root = make_patch_dir(str(tmp_path), per_fold=int(d["meta_per_fold"]), size=int(d["meta_size"]))
    sub = os.path.join(root, f"200x_{int(d['meta_size'])}")
    assert sorted(os.listdir(sub)) == [str(f) for f in d["files"]]
    for f, h in zip(d["files"], d["files_sha1"]):
        assert hashlib.sha1(open(os.path.join(sub, str(f)), "rb").read()).hexdigest() == str(h), f
    return d, root


def test_fold_splits_match_reference_fixture(tmp_path):
    """construct_train_valid / construct_test of the host side and of the oracle against the lists the
    reference's own utils/data_utils.py produced on the same directory (one fresh import per fold)."""
    d, root = _fixture_dir(tmp_path)
    for fold in (1, 2, 3, 4, 5):
        tr, va = D.construct_train_valid(root, test_fold=fold)
        otr, ova = OD.construct_train_valid(root, test_fold=fold)
        for got in ((tr, va), (otr, ova)):
            assert np.array_equal(got[0].astype(str), d[f"fold{fold}/train"]), fold
            assert np.array_equal(got[1].astype(str), d[f"fold{fold}/valid"]), fold
        assert np.array_equal(D.construct_test(root, test_fold=fold).astype(str), d[f"fold{fold}/test"])


def test_oracle_items_match_reference_fixture(tmp_path):
    """The oracle's PatchDataset.__getitem__ + Normalization [+ RandomFlip] + ToTensor restatement
    against the reference's own outputs for every item of fold 2 (flip draws as recorded): inputs
    bit-exact, labels equal (the reference's LongTensor values)."""
    d, root = _fixture_dir(tmp_path)
    for split, train in (("train", True), ("valid", False)):
        lst = d[f"fold2/{split}"]
        for i, (a, b) in enumerate(lst):
            inp, lab, pid = OD.read_patch(root, str(a), str(b), 200, int(d["meta_size"]))
            x, t = OD.transform(inp, lab, flips=int(d[f"{split}/flips"][i]), train=train)
            assert np.array_equal(x.view(np.uint32), d[f"{split}/input"][i].view(np.uint32)), (split, i)
            assert np.array_equal(t, d[f"{split}/label"][i].astype(np.float32)), (split, i)
            assert pid == str(d[f"{split}/ids"][i])
