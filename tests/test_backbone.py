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

from pvnet_amd.network import PVNet, PVNetInference, fold_batchnorm, upsample2x_cat
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


def test_inference_form_construction():
    """PVNetInference: convraw's first convolution is the folded one with 5
    zero input channels appended (the 35 -> 40 channel pad of the fused
    upsample + cat); no BatchNorm left."""
    net = _net()
    inf = PVNetInference(net)
    ref = fold_batchnorm(net).convraw[0]
    w = inf.convraw[0].weight
    assert w.shape == (32, 40, 3, 3)
    assert torch.equal(w[:, :35], ref.weight) and not w[:, 35:].any()
    assert torch.equal(inf.convraw[0].bias, ref.bias)
    assert not any(isinstance(m, torch.nn.BatchNorm2d) for m in inf.modules())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("c1,c2,cpad,h,w", [(32, 3, 40, 12, 16), (64, 64, 128, 7, 9), (128, 64, 192, 5, 6),
                                            (16, 0, 24, 3, 4)])
def test_upsample2x_cat_matches_torch(c1, c2, cpad, h, w, dtype, device):
    """The fused HIP decoder step equals ATen's UpsamplingBilinear2d + cat +
    zero pad on channels_last fp16 / f32 (the same f32 blend; fp16: at most one
    ulp; f32: a few roundings of the inputs' size, where the two compilers
    contract differently)."""
    g = torch.Generator().manual_seed(c1 + c2)
    cl = torch.channels_last
    fm = (torch.randn(3, c1, h, w, generator=g) * 4).to(device, dtype).contiguous(memory_format=cl)
    skip = (torch.randn(3, c2, 2 * h, 2 * w, generator=g) * 4).to(device, dtype).contiguous(memory_format=cl) \
        if c2 else None
    out = upsample2x_cat(fm, skip, cpad)
    up = torch.nn.UpsamplingBilinear2d(scale_factor=2)(fm)
    parts = [up] + ([skip] if c2 else [])
    ref = torch.cat(parts, 1)
    ref = torch.cat([ref, torch.zeros(3, cpad - ref.shape[1], 2 * h, 2 * w, dtype=ref.dtype, device=device)], 1)
    assert out.shape == ref.shape and out.is_contiguous(memory_format=cl)
    d = (out.float() - ref.float()).abs()
    if dtype == torch.float16:
        ulp = torch.clamp(ref.float().abs(), min=2 ** -14) * 2 ** -10
    else:   # f32: a few roundings of terms as large as the inputs (blends may cancel)
        ulp = torch.full_like(d, 4 * 2 ** -24 * float(fm.abs().max()))
    assert bool((d <= ulp).all()), float((d / ulp).max())
    assert torch.equal(out[:, c1:], ref[:, c1:])
    print(f"exact: {float((d == 0).float().mean()):.4f}")


@pytest.mark.gpu
def test_inference_form_device_fp16_matches_reference(device):
    """configs[2]'s backbone as the bench runs it (PVNetInference: folded BN,
    fused upsample + cat, fp16 channels_last) against G4: 1.5e-2 of scale."""
    net = PVNetInference(_net()).to(device=device, dtype=torch.float16).to(memory_format=torch.channels_last)
    x = torch.from_numpy(G["x_small"]).to(device).half().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
    sc = _scale()
    ds = np.abs(seg.float().cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.float().cpu().numpy() - G["ver_small"]).max()
    print(f"inference form fp16 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= 1.5e-2 * sc and dv <= 1.5e-2 * sc


@pytest.mark.gpu
def test_inference_form_device_fp32_matches_reference(device):
    """configs[1]'s backbone in the inference form, f32: 2e-4 of scale, as the
    plain module on MIOpen."""
    net = PVNetInference(_net()).to(device=device).to(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(G["x_small"]).to(device).contiguous(memory_format=torch.channels_last))
        fx = torch.from_numpy(BI.frame_input()).to(device).contiguous(memory_format=torch.channels_last)
        fseg, fver = net(fx)
    sc = _scale()
    ds = np.abs(seg.cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.cpu().numpy() - G["ver_small"]).max()
    print(f"inference form f32 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= 2e-4 * sc and dv <= 2e-4 * sc
    _frame_check(fseg.cpu().numpy(), fver.cpu().numpy(), 2e-4)
