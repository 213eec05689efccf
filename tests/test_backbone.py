"""Backbone parity, fixture G4: pvnet_amd.network.PVNet vs the
reference ``PVnet`` (lib/networks/model_repository.py:7-79 over
lib/networks/resnet.py:116-233).

tests/golden/backbone_g4.npz was made by tests/golden/make_golden_backbone.py,
which loaded the seeded state dict of tests/backbone_init.py into the
REFERENCE network with ``load_state_dict(strict=True)`` and recorded its
eval-mode fp32 outputs (torch-CPU).  Here the same seeded weights go into our
network:
  * CPU: key set + shapes equal the reference's (strict load both ways), the
    weights hash equals the fixture's, and the torch-CPU forward equals the
    reference's (same kernels, same order: tolerance 1e-5 of the output scale);
  * GPU (MIOpen): fp32 within 2e-4 of the output scale (different convolution
    algorithms sum in other orders), and fp16 + channels_last -- the
    configs[2] backbone -- within 1.5e-2 of the scale (the reference itself
    moves 2.9e-3 of scale in fp16 on CPU; ``f16_cpu_max_dev``).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from pvnet_amd.network import PVNet, fold_batchnorm
from tests import backbone_init as BI
from tests.golden_io import load

G = load("backbone_g4")


def _net(dtype=torch.float32, device="cpu", channels_last=False):
    net = PVNet(18, 2)
    sd = BI.seeded_state_dict(net.state_dict(), int(G["seed"]))
    assert BI.weights_sha(sd) == str(G["weights_sha"]), "seeded G4 weights drifted"
    net.load_state_dict(sd, strict=True)
    net = net.eval().to(device=device, dtype=dtype)
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    return net


def _scale():
    return float(max(np.abs(G["seg_small"]).max(), np.abs(G["ver_small"]).max()))


def _frame_check(seg, ver, tol):
    fs = BI.frame_summary(seg, ver)
    sc = float(np.abs(G["frame_lattice"]).max())
    assert np.abs(fs["lattice"] - G["frame_lattice"]).max() <= tol * sc
    assert np.abs(fs["window"] - G["frame_window"]).max() <= tol * sc
    np.testing.assert_allclose(fs["chan_sum"], G["frame_chan_sum"], rtol=tol * 10, atol=tol * sc * 480 * 640 * 1e-3)


def test_state_dict_keys_and_shapes_equal_reference():
    sd = PVNet(18, 2).state_dict()
    keys = sorted(sd)
    assert keys == [str(k) for k in G["keys"]]
    assert ["x".join(map(str, sd[k].shape)) for k in keys] == [str(s) for s in G["shapes"]]


def test_forward_cpu_matches_reference():
    net = _net()
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(G["x_small"]))
    sc = _scale()
    assert seg.shape == (1, 2, 64, 80) and ver.shape == (1, 18, 64, 80)
    assert np.abs(seg.numpy() - G["seg_small"]).max() <= 1e-5 * sc
    assert np.abs(ver.numpy() - G["ver_small"]).max() <= 1e-5 * sc


def test_forward_cpu_frame_matches_reference():
    net = _net()
    x = BI.frame_input()
    assert BI.sha(x) == str(G["frame_input_sha"])
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(x))
    _frame_check(seg.numpy(), ver.numpy(), 1e-5)


@pytest.mark.gpu
def test_forward_device_fp32_matches_reference(device):
    net = _net(device=device)
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(G["x_small"]).to(device))
        fseg, fver = net(torch.from_numpy(BI.frame_input()).to(device))
    sc = _scale()
    ds = np.abs(seg.cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.cpu().numpy() - G["ver_small"]).max()
    print(f"fp32 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= 2e-4 * sc and dv <= 2e-4 * sc
    _frame_check(fseg.cpu().numpy(), fver.cpu().numpy(), 2e-4)


@pytest.mark.gpu
def test_forward_device_fp16_channels_last_matches_reference(device):
    net = _net(dtype=torch.float16, device=device, channels_last=True)
    x = torch.from_numpy(G["x_small"]).to(device).half().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
    sc = _scale()
    ds = np.abs(seg.float().cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.float().cpu().numpy() - G["ver_small"]).max()
    print(f"fp16 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f} (reference fp16 on CPU: "
          f"{float(G['f16_cpu_max_dev']):.3e})")
    assert ds <= 1.5e-2 * sc and dv <= 1.5e-2 * sc


def test_folded_batchnorm_cpu_matches_reference():
    """fold_batchnorm (the bench's inference form): the seeded G4 weights
    carry non-trivial BN statistics; the folded forward equals the
    reference's outputs to 2e-5 of the scale (folding re-rounds the weights)."""
    net = fold_batchnorm(_net())
    assert sum(isinstance(m, torch.nn.BatchNorm2d) for m in _net().modules()) == 25
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(G["x_small"]))
    sc = _scale()
    assert np.abs(seg.numpy() - G["seg_small"]).max() <= 2e-5 * sc
    assert np.abs(ver.numpy() - G["ver_small"]).max() <= 2e-5 * sc


@pytest.mark.gpu
def test_folded_batchnorm_device_fp16_channels_last_matches_reference(device):
    """The configs[2] backbone as the bench runs it: BN folded, fp16,
    channels_last, on MIOpen -- within the same 1.5e-2 of scale as unfolded."""
    net = fold_batchnorm(_net()).to(device=device, dtype=torch.float16).to(memory_format=torch.channels_last)
    x = torch.from_numpy(G["x_small"]).to(device).half().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
        fseg, fver = fold_batchnorm(_net(device=device))(torch.from_numpy(BI.frame_input()).to(device))
    sc = _scale()
    ds = np.abs(seg.float().cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.float().cpu().numpy() - G["ver_small"]).max()
    print(f"folded fp16 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= 1.5e-2 * sc and dv <= 1.5e-2 * sc
    _frame_check(fseg.cpu().numpy(), fver.cpu().numpy(), 2e-4)
