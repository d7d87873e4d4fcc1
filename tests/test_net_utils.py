"""Checkpoint layout and interop (utils/net_utils.py:5-53, train.py:385) — CPU only."""
from collections import OrderedDict

import torch

import selectivenet_for_semantic_segmentation_binary_amd as S
from selectivenet_for_semantic_segmentation_binary_amd import net_utils as NU
from tests import _golden as G


def _net(seed):
    torch.manual_seed(seed)
    net = S.UNet_B("RGB", selective=True)
    with torch.no_grad():
        for p in net.parameters():
            p.normal_()
    return net


def test_state_dict_keys_are_the_references():
    net = S.UNet_B("RGB", selective=True)
    assert list(net.state_dict()) == G.kat()["state_dict_keys_selective"]
    heads = {"conv_select.weight", "conv_select.bias", "conv_aux.weight", "conv_aux.bias"}
    want = [k for k in G.kat()["state_dict_keys_selective"] if k not in heads]
    assert list(S.UNet_B("RGB", selective=False).state_dict()) == want


def test_save_resume_roundtrip_with_adam_state(tmp_path):
    net = _net(0)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    for p in net.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    for e in (2, 10, 9):
        NU.net_save(str(tmp_path), net, opt, e)
    net2 = _net(1)
    opt2 = S.Adam(net2.parameters(), lr=1e-3)
    net2, opt2, epoch = NU.net_train_load(str(tmp_path), net2, opt2)
    assert epoch == 10  # newest by the digits in the name, as the reference sorts
    for (k, a), (_, b) in zip(net.state_dict().items(), net2.state_dict().items()):
        assert torch.equal(a, b), k
    s1, s2 = opt.state_dict(), opt2.state_dict()
    assert s1["param_groups"][0]["params"] == s2["param_groups"][0]["params"]
    for i in s1["state"]:
        assert torch.equal(s1["state"][i]["exp_avg"], s2["state"][i]["exp_avg"])
        assert torch.equal(s1["state"][i]["exp_avg_sq"], s2["state"][i]["exp_avg_sq"])


def test_dataparallel_prefixed_checkpoint_loads(tmp_path):
    net = _net(3)
    sd = OrderedDict(("module." + k, v) for k, v in net.state_dict().items())
    torch.save({"net": sd, "optim": {}}, tmp_path / "model_epoch1.pth")
    net2 = NU.net_test_load(str(tmp_path / "model_epoch1.pth"), _net(4))
    for (k, a), (_, b) in zip(net.state_dict().items(), net2.state_dict().items()):
        assert torch.equal(a, b), k


def test_missing_dir_starts_at_epoch_zero(tmp_path):
    net = _net(0)
    opt = S.Adam(net.parameters())
    assert NU.net_train_load(str(tmp_path / "nope"), net, opt)[2] == 0
