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
    configs[2] backbone -- within 1e-2 of the scale (the reference itself
    moves 2.9e-3 of scale in fp16 on CPU; ``f16_cpu_max_dev``).
  * the full-frame segmentation masks (argmax(seg_pred, 1), the north
    star's "segmentation masks bit-exact") against the reference's, for
    PVnet(18, 2) and configs[4]'s PVnet(42, 2) (fixture backbone_g4_masks).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from pvnet_amd.network import PVNet, PVNetInference, fold_batchnorm, upsample2x_cat
from tests import backbone_init as BI
from tests import fp16_bounds as B
from tests.golden_io import load

G = load("backbone_g4")
# fp16 device tolerance (of the output scale): measured 3.7e-3 .. 6.8e-3 on the
# G4 weights (plain, folded, inference form; PVnet(42, 2) 2.7e-3 / 3.7e-3); the
# reference's own fp16 forward on CPU moves 2.9e-3 (f16_cpu_max_dev)
FP16_TOL = 1e-2


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
    assert ds <= FP16_TOL * sc and dv <= FP16_TOL * sc


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
    channels_last, on MIOpen -- within the same FP16_TOL of scale as unfolded."""
    net = fold_batchnorm(_net()).to(device=device, dtype=torch.float16).to(memory_format=torch.channels_last)
    x = torch.from_numpy(G["x_small"]).to(device).half().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
        fseg, fver = fold_batchnorm(_net(device=device))(torch.from_numpy(BI.frame_input()).to(device))
    sc = _scale()
    ds = np.abs(seg.float().cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.float().cpu().numpy() - G["ver_small"]).max()
    print(f"folded fp16 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= FP16_TOL * sc and dv <= FP16_TOL * sc
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
    fused upsample + cat, fp16 channels_last) against G4: FP16_TOL of scale."""
    net = PVNetInference(_net()).to(device=device, dtype=torch.float16).to(memory_format=torch.channels_last)
    x = torch.from_numpy(G["x_small"]).to(device).half().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
    sc = _scale()
    ds = np.abs(seg.float().cpu().numpy() - G["seg_small"]).max()
    dv = np.abs(ver.float().cpu().numpy() - G["ver_small"]).max()
    print(f"inference form fp16 device: max dev {ds:.3e} / {dv:.3e} of scale {sc:.2f}")
    assert ds <= FP16_TOL * sc and dv <= FP16_TOL * sc


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


# ---------------------------------------------------------------- segmentation masks (north star: bit-exact)
GM = load("backbone_g4_masks")


def _mask_net(vd, dtype=torch.float32, device="cpu", form="plain"):
    """PVNet(vd, 2) with the mask fixture's weights (G4's seeded weights, the
    foreground bias shifted by the stored amount: half the frame is
    foreground)."""
    net = PVNet(vd, 2)
    sd = BI.mask_state_dict(net.state_dict(), float(GM[f"shift_{vd}"]))
    assert BI.weights_sha(sd) == str(GM[f"weights_sha_{vd}"]), "mask fixture weights drifted"
    net.load_state_dict(sd, strict=True)
    net = net.eval()
    if form == "inference":
        net = PVNetInference(net)
    net = net.to(device=device, dtype=dtype)
    if form == "inference" or dtype == torch.float16:
        net = net.to(memory_format=torch.channels_last)
    return net


def _frame(device="cpu", dtype=torch.float32, channels_last=False):
    x = BI.frame_input()
    assert BI.sha(x) == str(GM["frame_input_sha"])
    t = torch.from_numpy(x).to(device=device, dtype=dtype)
    return t.contiguous(memory_format=torch.channels_last) if channels_last else t


def _mask_compare(seg, vd, band):
    """Compare argmax(seg, 1) (first index on ties) with the reference's mask.
    Returns (mismatching pixels, how many of them lie outside the reference's
    stored low-margin set, pixels whose own margin is within `band`)."""
    seg = seg.float().cpu().numpy()
    got = (seg[0, 1] > seg[0, 0]).ravel()
    want = np.unpackbits(GM[f"mask_bits_{vd}"])[: got.size].astype(bool)
    diff = np.nonzero(got != want)[0]
    outside = np.setdiff1d(diff, GM[f"margin_idx_{vd}"])
    d_own = (seg[0, 1] - seg[0, 0]).ravel()
    return diff, outside, d_own


def test_mask_fixture_matches_reference_mask_counts():
    """The fixture's masks are the reference's (half-frame foreground) and
    the low-margin sets are small: the bit-exact claim covers the rest."""
    for vd in (18, 42):
        bits = np.unpackbits(GM[f"mask_bits_{vd}"])[: 480 * 640]
        assert int(bits.sum()) == int(GM[f"fg_count_{vd}"])
        assert 0.45 < bits.mean() < 0.55
        assert GM[f"margin_idx_{vd}"].size < 0.01 * bits.size


@pytest.mark.parametrize("vd", [18, 42])
def test_segmentation_mask_cpu_bit_exact(vd):
    """torch-CPU forward of our PVNet(vd, 2): the full-frame argmax mask equals
    the reference's everywhere (outside the < 4e-4-of-scale margin set any
    difference would fail)."""
    with torch.no_grad():
        seg, _ = _mask_net(vd)(_frame())
    diff, outside, _ = _mask_compare(seg, vd, 0)
    print(f"PVNet({vd},2) CPU mask: {diff.size} differing pixels ({outside.size} outside the margin set)")
    assert outside.size == 0


def test_pvnet42_cpu_matches_reference():
    """configs[4]'s head, PVnet(42, 2) (MR:57 ver_dim sets the last conv):
    key/shape equality with the reference (strict load of the fixture's
    weights) and the CPU forward within 1e-5 of scale, small input and frame."""
    net = _mask_net(42)
    assert tuple(net.convraw[3].weight.shape) == (44, 32, 1, 1)
    with torch.no_grad():
        seg, ver = net(torch.from_numpy(G["x_small"]))
        fseg, fver = net(_frame())
    sc = float(max(np.abs(GM["seg_small_42"]).max(), np.abs(GM["ver_small_42"]).max()))
    assert np.abs(seg.numpy() - GM["seg_small_42"]).max() <= 1e-5 * sc
    assert np.abs(ver.numpy() - GM["ver_small_42"]).max() <= 1e-5 * sc
    fs = BI.frame_summary(fseg.numpy(), fver.numpy())
    fsc = float(np.abs(GM["frame_lattice_42"]).max())
    assert np.abs(fs["lattice"] - GM["frame_lattice_42"]).max() <= 1e-5 * fsc
    assert np.abs(fs["window"] - GM["frame_window_42"]).max() <= 1e-5 * fsc


@pytest.mark.gpu
@pytest.mark.parametrize("vd", [18, 42])
@pytest.mark.parametrize("form", ["plain", "inference"])
def test_segmentation_mask_device_fp32_bit_exact(vd, form, device):
    """configs[1]'s fp32 forward on MIOpen (the plain module and the inference
    form): the full 480x640 argmax mask equals the reference's at every pixel
    outside the fixture's margin set (|l1 - l0| < 4e-4 of scale, twice the fp32
    device tolerance); the count of differing pixels is printed."""
    with torch.no_grad():
        seg, ver = _mask_net(vd, device=device, form=form)(_frame(device, channels_last=form == "inference"))
    diff, outside, _ = _mask_compare(seg, vd, 0)
    print(f"PVNet({vd},2) {form} fp32 device mask: {diff.size} differing pixels of {480 * 640} "
          f"({GM[f'margin_idx_{vd}'].size} in the margin set), {outside.size} outside it")
    assert outside.size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("vd", [18, 42])
def test_segmentation_mask_device_fp16(vd, device):
    """configs[2]/[4]'s fp16 inference-form forward: the mask's differing
    pixels are counted and reported, and each one is a near-tie -- its own
    logit margin is within the fp16 deviation bound 2 x FP16_TOL of scale, so
    the reference and the fp16 forward may resolve it either way.  The
    consequence for voting is reported too: the angle between the fp16 and
    the fp32 device vertex directions on the foreground (the fp32 forward is
    within 2e-4 of the reference's), against the 0.1415 rad cone of
    inlier_thresh 0.99."""
    net = _mask_net(vd, dtype=torch.float16, device=device, form="inference")
    net32 = _mask_net(vd, device=device, form="inference")
    with torch.no_grad():
        seg, ver = net(_frame(device, torch.float16, channels_last=True))
        _, ver32 = net32(_frame(device, channels_last=True))
    diff, outside, d_own = _mask_compare(seg, vd, 0)
    sc = float(GM[f"scale_{vd}"])
    fg = np.unpackbits(GM[f"mask_bits_{vd}"])[: 480 * 640].reshape(480, 640).astype(bool)
    v16 = ver.float().cpu().numpy()[0].reshape(vd // 2, 2, 480, 640)[:, :, fg]
    v32 = ver32.cpu().numpy()[0].reshape(vd // 2, 2, 480, 640)[:, :, fg]
    ang = np.abs(np.arctan2(v16[:, 1], v16[:, 0]) - np.arctan2(v32[:, 1], v32[:, 0]))
    ang = np.minimum(ang, 2 * np.pi - ang)
    print(f"PVNet({vd},2) fp16 inference device mask: {diff.size} differing pixels of {480 * 640} "
          f"({outside.size} outside the fp32 margin set); largest own margin among them "
          f"{float(np.abs(d_own[diff]).max()) if diff.size else 0.0:.4f} (scale {sc:.1f}, bound "
          f"{2 * FP16_TOL * sc:.3f}); vertex direction vs fp32: median {np.median(ang):.2e}, "
          f"p99 {np.quantile(ang, 0.99):.2e}, max {ang.max():.2e} rad")
    assert np.all(np.abs(d_own[diff]) <= 2 * FP16_TOL * sc)
    # measured 0.8 % (PVnet(18, 2)) and 2.4 % (PVnet(42, 2)) of the frame
    # (DESIGN.md 3); the gate is that count plus a quarter
    assert diff.size <= {18: 0.012, 42: 0.03}[vd] * d_own.size


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_pvnet42_device_matches_reference(dtype, device):
    """PVnet(42, 2) -- configs[4]'s backbone head -- on the device, inference
    form: small input and frame summary against the reference (fp32 2e-4,
    fp16 6e-3 of scale)."""
    net = _mask_net(42, dtype=dtype, device=device, form="inference")
    x = torch.from_numpy(G["x_small"]).to(device=device, dtype=dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        seg, ver = net(x)
        fseg, fver = net(_frame(device, dtype, channels_last=True))
    tol = 2e-4 if dtype == torch.float32 else FP16_TOL
    sc = float(max(np.abs(GM["seg_small_42"]).max(), np.abs(GM["ver_small_42"]).max()))
    ds = np.abs(seg.float().cpu().numpy() - GM["seg_small_42"]).max()
    dv = np.abs(ver.float().cpu().numpy() - GM["ver_small_42"]).max()
    print(f"PVNet(42,2) {dtype} device: max dev {ds / sc:.3e} / {dv / sc:.3e} of scale")
    assert ds <= tol * sc and dv <= tol * sc
    fs = BI.frame_summary(fseg.float().cpu().numpy(), fver.float().cpu().numpy())
    fsc = float(np.abs(GM["frame_lattice_42"]).max())
    assert np.abs(fs["lattice"] - GM["frame_lattice_42"]).max() <= tol * fsc
    assert np.abs(fs["window"] - GM["frame_window_42"]).max() <= tol * fsc


# ---------------------------------------------------------------- fused epilogues of the inference form
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("case", ["relu", "leaky", "residual", "residual_rbias", "cat"])
def test_conv_epilogue_matches_torch(case, dtype, device):
    """pv_conv_epilogue equals ATen's unfused ops on the same channels-last
    conv output bit for bit: y + bias, (+ (res + rbias)), ReLU / LeakyReLU(0.1),
    and the torch.cat([.., skip], 1) after fc."""
    from pvnet_amd.network import conv_epilogue
    g = torch.Generator().manual_seed(hash(case) % 1000)
    cl = torch.channels_last
    n, c, h, w = 3, 64, 9, 13
    y = (torch.randn(n, c, h, w, generator=g) * 3).to(device, dtype).contiguous(memory_format=cl)
    b = (torch.randn(c, generator=g)).to(device, dtype)
    res = (torch.randn(n, c, h, w, generator=g) * 3).to(device, dtype).contiguous(memory_format=cl)
    rb = (torch.randn(c, generator=g)).to(device, dtype)
    skip = (torch.randn(n, 32, h, w, generator=g)).to(device, dtype).contiguous(memory_format=cl)
    ref = y + b.view(1, -1, 1, 1)
    if case.startswith("residual"):
        ref = ref + ((res + rb.view(1, -1, 1, 1)) if case.endswith("rbias") else res)
    ref = torch.nn.functional.leaky_relu(ref, 0.1) if case == "leaky" else torch.relu(ref)
    if case == "cat":
        ref = torch.cat([ref, skip], 1)
    got = conv_epilogue(y.clone(memory_format=cl), b, "leaky" if case == "leaky" else "relu",
                        res=res if case.startswith("residual") else None,
                        rbias=rb if case == "residual_rbias" else None, skip=skip if case == "cat" else None)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    assert torch.equal(got, ref.contiguous(memory_format=cl))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("cout", [20, 44])
def test_head_matches_torch(cout, dtype, device):
    """pv_head (convraw's bias + LeakyReLU + 1x1 convolution + bias, MR:53-58)
    against ATen's modules on the same input: the activation bit for bit,
    the 1x1 sum within a few roundings (MIOpen sums in another order)."""
    from pvnet_amd.network import head
    g = torch.Generator().manual_seed(cout)
    cl = torch.channels_last
    y = (torch.randn(2, 32, 24, 40, generator=g) * 2).to(device, dtype).contiguous(memory_format=cl)
    b1 = torch.randn(32, generator=g).to(device, dtype)
    conv = torch.nn.Conv2d(32, cout, 1).to(device, dtype)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, 32, 1, 1, generator=g) * 0.3)
        conv.bias.copy_(torch.randn(cout, generator=g))
        t = torch.nn.functional.leaky_relu(y + b1.view(1, -1, 1, 1), 0.1)
        ref = conv(t)
        got = head(y, b1.float(), conv.weight.float().reshape(cout, 32), conv.bias.float(), 0.1)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(t.abs().max()) * float(conv.weight.abs().sum(1).max())
    tol = (2 ** -10 if dtype == torch.float16 else 2 ** -20) * sc
    d = (got.float() - ref.float()).abs().max()
    print(f"head {dtype} cout {cout}: max dev {float(d):.3e} (tolerance {tol:.3e})")
    assert float(d) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("cout", [20, 44])
@pytest.mark.parametrize("hw", [(13, 21, 2), (60, 80, 2), (120, 160, 8)])
def test_decoder_tail_matches_torch(cout, hw, device):
    """pv_decoder_tail_f16 (up2storaw + cat([fm, x]) + convraw, MR:75-79, one
    matrix-core pass) against ATen's unfused fp16 ops on the same inputs:
    F.interpolate + torch.cat + the 3x3 conv + bias + LeakyReLU + the 1x1
    conv.  Both sum in f32 and round the 3x3 output to fp16 (MIOpen in
    another order), so the outputs agree within a couple of fp16 roundings
    of the head's scale; ragged tiles (13 x 21 -> 26 x 42) included.  The
    batch-8 case has 2,400 tiles for the 3 x CUs persistent blocks, so every
    block runs several tiles: the next tile's patch and image rows land in
    LDS (buffer loads to LDS) while the block convolves the current one."""
    from pvnet_amd.network import decoder_tail, decoder_tail_weights
    F = torch.nn.functional
    g = torch.Generator().manual_seed(cout + hw[0])
    cl = torch.channels_last
    h, w, n = hw
    fm = (torch.randn(n, 32, h, w, generator=g) * 2).to(device, torch.float16).contiguous(memory_format=cl)
    img = torch.randn(n, 3, 2 * h, 2 * w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    c0 = torch.nn.Conv2d(35, 32, 3, 1, 1).to(device)
    c1 = torch.nn.Conv2d(32, cout, 1).to(device)
    with torch.no_grad():
        c0.weight.copy_(torch.randn(32, 35, 3, 3, generator=g) * 0.1)
        c0.bias.copy_(torch.randn(32, generator=g) * 0.5)
        c1.weight.copy_(torch.randn(cout, 32, 1, 1, generator=g) * 0.3)
        c1.bias.copy_(torch.randn(cout, generator=g))
        c0, c1 = c0.half(), c1.half()
        up = F.interpolate(fm, scale_factor=2, mode="bilinear", align_corners=True)
        t = F.leaky_relu(F.conv2d(torch.cat([up, img], 1), c0.weight, None, 1, 1) + c0.bias.view(1, -1, 1, 1), 0.1)
        ref = c1(t)
        got = decoder_tail(fm, img, decoder_tail_weights(c0, c1), 0.1)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(t.abs().max()) * float(c1.weight.float().abs().sum((1, 2, 3)).max())
    tol = 2 ** -9 * sc
    d = (got.float() - ref.float()).abs()
    print(f"decoder tail cout {cout} {2 * h}x{2 * w}: max dev {float(d.max()):.3e}, "
          f"mean {float(d.mean()):.3e} (tolerance {tol:.3e}, scale {sc:.2f})")
    assert float(d.max()) <= tol
    assert float(d.mean()) <= 2 ** -12 * sc
    _check_decoder_fp64(got, fm, img, c0, 0.1, f"decoder tail cout {cout}", head=(c1.weight, c1.bias))
    # the split form (pv_decoder_tail_split_f16): seg and ver as two dense
    # channels_last maps, bit-equal to the one-buffer form's channel slices
    with torch.no_grad():
        seg, ver = decoder_tail(fm, img, decoder_tail_weights(c0, c1), 0.1, split=True)
    torch.cuda.synchronize()
    assert seg.shape == (n, 2, 2 * h, 2 * w) and ver.shape == (n, cout - 2, 2 * h, 2 * w)
    assert seg.is_contiguous(memory_format=cl) and ver.is_contiguous(memory_format=cl)
    assert torch.equal(seg, got[:, :2]) and torch.equal(ver, got[:, 2:])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("hw", [(24, 40), (23, 17)])
def test_relu_maxpool_matches_torch(dtype, hw, device):
    """pv_relu_maxpool (the stem's bias + ReLU = x2s and maxpool 3x3/2/1,
    RN:201-204) equals ATen's ops bit for bit, odd sizes included."""
    from pvnet_amd.network import relu_maxpool
    g = torch.Generator().manual_seed(hw[0] * 100 + hw[1])
    cl = torch.channels_last
    y = (torch.randn(3, 64, *hw, generator=g) * 3).to(device, dtype).contiguous(memory_format=cl)
    b = torch.randn(64, generator=g).to(device, dtype)
    ref_x2s = torch.relu(y + b.view(1, -1, 1, 1))
    ref_pool = torch.nn.functional.max_pool2d(ref_x2s, 3, 2, 1)
    x2s, pool = relu_maxpool(y, b)
    assert x2s.is_contiguous(memory_format=cl) and pool.is_contiguous(memory_format=cl)
    assert torch.equal(x2s, ref_x2s) and torch.equal(pool, ref_pool)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("hw", [(240, 320), (37, 51), (10, 7), (3, 2)])
def test_maxpool_matches_torch(dtype, hw, device):
    """The pool-only form of pv_relu_maxpool (the stem kernel's maxpool,
    RN:204) is bit-equal to ATen's max_pool2d(3, 2, 1), odd and tiny maps
    included."""
    from pvnet_amd.network import maxpool
    g = torch.Generator().manual_seed(hw[0] * 100 + hw[1])
    cl = torch.channels_last
    x = torch.randn(2, 64, *hw, generator=g).to(device, dtype).contiguous(memory_format=cl)
    got = maxpool(x)
    ref = torch.nn.functional.max_pool2d(x, 3, 2, 1)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["relu_128_256_d2", "res_256_256_d2", "resb_256_512_d4", "relu_512_512_d4",
                                  "fc_512_256_d1_ragged", "leaky_64_256_d1", "resb_128_128_d1",
                                  "leaky_384_128_d1_ragged", "resb_256_512_d4_big", "relu_128_128_d1_big"])
def test_conv3x3_matches_torch(case, device):
    """pv_conv3x3_f16 (the wide 3x3 convolutions of layer3 / layer4 / fc with
    their epilogue, RN:21-38 / MR:22-26) against MIOpen's fp16 convolution +
    ATen's bias / residual / activation on the same inputs.  Both sum in f32
    and round the convolution to fp16 (in other orders), so the outputs agree
    within a couple of fp16 roundings of the convolution's scale; padding,
    dilation, a pixel count that is not a multiple of the tile and the
    128-cout tiles (layer2, conv8s) included."""
    from pvnet_amd.network import conv3x3, conv3x3_weight
    F = torch.nn.functional
    kind, cin, cout, d = case.split("_")[0], *[int(v) for v in case.split("_")[1:3]], int(case.split("_")[3][1:])
    # "big": more tiles than CUs, so whole tiles run beside the split last round
    n, h, w = (3, 13, 17) if case.endswith("ragged") else (16, 60, 80) if case.endswith("big") else (2, 30, 40)
    g = torch.Generator().manual_seed(cin * 7 + cout + d)
    cl = torch.channels_last
    x = torch.randn(n, cin, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    conv = torch.nn.Conv2d(cin, cout, 3, 1, d, d, bias=True).to(device)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.5)
    conv = conv.half()
    res = torch.randn(n, cout, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    rb = (torch.randn(cout, generator=g) * 0.5).to(device, torch.float16)
    use_res, use_rb = kind in ("res", "resb"), kind == "resb"
    act = "leaky" if kind == "leaky" else "relu"
    with torch.no_grad():
        y = F.conv2d(x, conv.weight, None, 1, d, d) + conv.bias.view(1, -1, 1, 1)
        if use_res:
            y = y + ((res + rb.view(1, -1, 1, 1)) if use_rb else res)
        ref = F.leaky_relu(y, 0.1) if act == "leaky" else torch.relu(y)
        got = conv3x3(x, conv3x3_weight(conv), conv.bias, d, act, res=res if use_res else None,
                      rbias=rb if use_rb else None)
        again = conv3x3(x, conv3x3_weight(conv), conv.bias, d, act, res=res if use_res else None,
                        rbias=rb if use_rb else None)
    torch.cuda.synchronize()
    assert torch.equal(got, again)          # split tiles sum their parts in part order, whatever arrives last
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    dev_ = (got.float() - ref.float()).abs()
    print(f"conv3x3 {case}: max dev {float(dev_.max()):.3e}, mean {float(dev_.mean()):.2e} (scale {sc:.2f})")
    assert float(dev_.max()) <= 2 ** -8 * sc
    assert float(dev_.mean()) <= 2 ** -13 * sc
    # against an f64 convolution of the same fp16 inputs: only the f32
    # accumulation and the epilogue's fp16 roundings (tests/fp16_bounds.py)
    with torch.no_grad():
        c64 = B.conv64(x, conv.weight, padding=d, dilation=d)
        e = B.round_step(c64, B.acc_bound(x, conv.weight, 9 * cin, padding=d, dilation=d))   # fp16 conv output
        y64 = c64 + conv.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)                                                               # + bias
        if use_res:
            r64 = res.double() + (rb.double().view(1, -1, 1, 1) if use_rb else 0.0)
            if use_rb:
                e = e + B.hulp(r64)                                                            # res + rbias
            y64 = y64 + r64
            e = B.round_step(y64, e)                                                           # + residual
        if act == "leaky":
            e = B.leaky_step(y64, e, 0.1)
            y64 = F.leaky_relu(y64, 0.1)
        else:
            y64 = torch.relu(y64)
    B.check(got, y64, e, f"conv3x3 {case}")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["s2_64_128_d1", "s2_64_128_d1_odd", "cat_256_128_d1", "cat_256_128_d1_ragged",
                                  "ds1_128_256_d2", "ds2_64_128_d1", "ds2_64_128_d1_odd", "ds1_256_512_d4"])
def test_conv3x3_ex_matches_torch(case, device):
    """pv_conv3x3_ex_f16 against MIOpen's fp16 convolutions + ATen's epilogue
    on the same inputs: "s2" layer2's stride-2 first convolution (RN:167-198);
    "cat" conv8s over torch.cat([xfc, x8s], 1) read from the two maps (MR:66);
    "ds1" / "ds2" a BasicBlock's conv2 with its 1x1 downsample (stride 1 / 2)
    summed into the same accumulator, then bias, the downsample's bias and the
    ReLU (RN:41-70).  Odd input sizes (stride 2) and a ragged pixel count
    included.  Tolerance as test_conv3x3_matches_torch (the fused sum skips
    the reference's fp16 roundings of the two convolutions)."""
    from pvnet_amd.network import conv3x3_ex, conv3x3_weight
    F = torch.nn.functional
    parts = case.split("_")
    kind, cin, cout, d = parts[0], int(parts[1]), int(parts[2]), int(parts[3][1:])
    n, h, w = (3, 13, 17) if case.endswith("ragged") else (2, 31, 41) if case.endswith("odd") else (2, 30, 40)
    g = torch.Generator().manual_seed(cin * 11 + cout + d + len(case))
    cl = torch.channels_last

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g) * scale).to(device, torch.float16)

    def conv_w(co, ci, k):
        return rnd(co, ci, k, k, scale=1.0 / (k * ci ** 0.5))

    b = rnd(cout, scale=0.5)
    with torch.no_grad():
        if kind == "s2":
            x = rnd(n, cin, h, w).contiguous(memory_format=cl)
            wt = conv_w(cout, cin, 3)
            ref = torch.relu(F.conv2d(x, wt, None, 2, d, d) + b.view(1, -1, 1, 1))
            c = torch.nn.Conv2d(cin, cout, 3, 2, d, d).to(device).half()
            c.weight.copy_(wt)
            got = conv3x3_ex(x, conv3x3_weight(c), b, d, stride=2, act="relu")
        elif kind == "cat":
            c2 = 128
            x = rnd(n, cin, h, w).contiguous(memory_format=cl)
            x2 = rnd(n, c2, h, w).contiguous(memory_format=cl)
            wt = conv_w(cout, cin + c2, 3)
            ref = F.leaky_relu(F.conv2d(torch.cat([x, x2], 1), wt, None, 1, d, d) + b.view(1, -1, 1, 1), 0.1)
            c = torch.nn.Conv2d(cin + c2, cout, 3, 1, d, d).to(device).half()
            c.weight.copy_(wt)
            got = conv3x3_ex(x, conv3x3_weight(c), b, d, act="leaky", x2=x2, mode2="cat")
        else:
            s2 = int(kind[2])
            cmid = cout
            xin = rnd(n, cin, h, w).contiguous(memory_format=cl)           # the block input
            ho, wo = (h - 1) // s2 + 1, (w - 1) // s2 + 1
            y = rnd(n, cmid, ho, wo).contiguous(memory_format=cl)          # conv1's output
            wt = conv_w(cout, cmid, 3)
            wd = conv_w(cout, cin, 1)
            bd = rnd(cout, scale=0.5)
            main = F.conv2d(y, wt, None, 1, d, d) + b.view(1, -1, 1, 1)
            resid = F.conv2d(xin, wd, None, s2) + bd.view(1, -1, 1, 1)
            ref = torch.relu(main + resid)
            c = torch.nn.Conv2d(cmid, cout, 3, 1, d, d).to(device).half()
            c.weight.copy_(wt)
            ds = torch.nn.Conv2d(cin, cout, 1, s2).to(device).half()
            ds.weight.copy_(wd)
            got = conv3x3_ex(y, conv3x3_weight(c, ds), b, d, act="relu", x2=xin, mode2="1x1", s2=s2, rbias=bd)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    dev_ = (got.float() - ref.float()).abs()
    print(f"conv3x3_ex {case}: max dev {float(dev_.max()):.3e}, mean {float(dev_.mean()):.2e} (scale {sc:.2f})")
    assert float(dev_.max()) <= 2 ** -8 * sc
    assert float(dev_.mean()) <= 2 ** -13 * sc
    # against an f64 convolution of the same fp16 inputs (tests/fp16_bounds.py):
    # the 1x1 downsample is summed in the same accumulator, rounded once
    with torch.no_grad():
        if kind == "s2":
            c64 = B.conv64(x, wt, stride=2, padding=d, dilation=d)
            e = B.acc_bound(x, wt, 9 * cin, stride=2, padding=d, dilation=d)
        elif kind == "cat":
            xc = torch.cat([x, x2], 1)
            c64 = B.conv64(xc, wt, padding=d, dilation=d)
            e = B.acc_bound(xc, wt, 9 * (cin + c2), padding=d, dilation=d)
        else:
            c64 = B.conv64(y, wt, padding=d, dilation=d) + B.conv64(xin, wd, stride=s2)
            e = B.acc_bound(y, wt, 9 * cmid + cin, padding=d, dilation=d) + \
                B.acc_bound(xin, wd, 9 * cmid + cin, stride=s2)
        e = B.round_step(c64, e)
        y64 = c64 + b.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)
        if kind.startswith("ds"):
            y64 = y64 + bd.double().view(1, -1, 1, 1)
            e = B.round_step(y64, e)
        if kind == "cat":
            e = B.leaky_step(y64, e, 0.1)
            y64 = F.leaky_relu(y64, 0.1)
        else:
            y64 = torch.relu(y64)
    B.check(got, y64, e, f"conv3x3_ex {case}")


def test_conv3x3_weight_with_downsample():
    """The PV_CONV_X2_1X1 weight rows: conv2's [cout][3][3][cmid] flattened,
    then the 1x1 downsample's [cout][cin] (include/pvvote.h)."""
    from pvnet_amd.network import conv3x3_weight
    c = torch.nn.Conv2d(128, 256, 3, 1, 1)
    ds = torch.nn.Conv2d(64, 256, 1, 2)
    w = conv3x3_weight(c, ds).float()
    assert tuple(w.shape) == (256, 9 * 128 + 64)
    ref_main = c.weight.detach().permute(0, 2, 3, 1).reshape(256, -1).half().float()
    assert torch.equal(w[:, :9 * 128], ref_main)
    assert torch.equal(w[:, 9 * 128:], ds.weight.detach().reshape(256, 64).half().float())


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(13, 21, 2), (60, 80, 2), (60, 80, 8)])
def test_decoder_conv2s_matches_torch(hw, device):
    """pv_decoder_conv2s_f16 (up4sto2s + cat([fm, x2s]) + conv2s, MR:43-51, one
    matrix-core pass) against ATen's unfused fp16 ops on the same inputs:
    F.interpolate + torch.cat + the 3x3 conv + bias + LeakyReLU.  The blend's
    fp16 weights and the summation order differ, so the outputs agree within
    a couple of fp16 roundings of the convolution's scale; ragged tiles
    (26 x 42) included; batch 8 at 120 x 160 has more tiles than persistent
    blocks (the next tile's inputs prefetched during a tile)."""
    from pvnet_amd.network import decoder_conv2s, decoder_conv2s_weights
    F = torch.nn.functional
    g = torch.Generator().manual_seed(hw[0] * 31 + hw[1])
    cl = torch.channels_last
    h, w, n = hw
    fm = (torch.randn(n, 64, h, w, generator=g) * 2).to(device, torch.float16).contiguous(memory_format=cl)
    skip = torch.randn(n, 64, 2 * h, 2 * w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    c = torch.nn.Conv2d(128, 32, 3, 1, 1).to(device)
    with torch.no_grad():
        c.weight.copy_(torch.randn(32, 128, 3, 3, generator=g) * 0.05)
        c.bias.copy_(torch.randn(32, generator=g) * 0.5)
    c = c.half()
    with torch.no_grad():
        up = F.interpolate(fm, scale_factor=2, mode="bilinear", align_corners=True)
        y = F.conv2d(torch.cat([up, skip], 1), c.weight, None, 1, 1) + c.bias.view(1, -1, 1, 1)
        ref = F.leaky_relu(y, 0.1)
        got = decoder_conv2s(fm, skip, decoder_conv2s_weights(c), 0.1)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    d = (got.float() - ref.float()).abs()
    print(f"decoder conv2s {2 * h}x{2 * w}: max dev {float(d.max()):.3e}, mean {float(d.mean()):.2e} (scale {sc:.2f})")
    assert float(d.max()) <= 2 ** -7 * sc
    assert float(d.mean()) <= 2 ** -12 * sc
    _check_decoder_fp64(got, fm, skip, c, 0.1, "decoder conv2s")


def test_decoder_conv_weight_layouts():
    """The host-side weight images of pv_decoder_conv2s_f16 / _conv4s_f16
    follow include/pvvote.h's index formulas (CPU)."""
    from pvnet_amd.network import decoder_conv2s_weights, decoder_conv4s_weights
    g = torch.Generator().manual_seed(5)
    c4 = torch.nn.Conv2d(192, 64, 3, 1, 1)
    c2 = torch.nn.Conv2d(128, 32, 3, 1, 1)
    with torch.no_grad():
        c4.weight.copy_(torch.randn(64, 192, 3, 3, generator=g))
        c2.weight.copy_(torch.randn(32, 128, 3, 3, generator=g))
    w4, _ = decoder_conv4s_weights(c4)
    w2, _ = decoder_conv2s_weights(c2)
    W4, W2 = c4.weight.detach().half(), c2.weight.detach().half()
    for p in range(3):
        for tap in range(9):
            for q in range(8):
                blk = W4[:, 64 * p + 8 * q: 64 * p + 8 * q + 8, tap // 3, tap % 3]          # [64, 8]
                assert torch.equal(w4[p, tap, q].reshape(64, 8), blk)
    for p in range(2):
        for tap in range(9):
            for q in range(8):
                assert torch.equal(w2[p, tap, q], W2[:, 64 * p + 8 * q: 64 * p + 8 * q + 8, tap // 3, tap % 3])


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(13, 21, 2), (60, 80, 2), (60, 80, 8)])
def test_decoder_conv4s_matches_torch(hw, device):
    """pv_decoder_conv4s_f16 (up8sto4s + cat([fm, x4s]) + conv4s, MR:35-43)
    against ATen's unfused fp16 ops; tolerance as the conv2s test (batch 8:
    several tiles per persistent block)."""
    from pvnet_amd.network import decoder_conv4s, decoder_conv4s_weights
    F = torch.nn.functional
    g = torch.Generator().manual_seed(hw[0] * 17 + hw[1])
    cl = torch.channels_last
    h, w, n = hw
    fm = (torch.randn(n, 128, h, w, generator=g) * 2).to(device, torch.float16).contiguous(memory_format=cl)
    skip = torch.randn(n, 64, 2 * h, 2 * w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    c = torch.nn.Conv2d(192, 64, 3, 1, 1).to(device)
    with torch.no_grad():
        c.weight.copy_(torch.randn(64, 192, 3, 3, generator=g) * 0.04)
        c.bias.copy_(torch.randn(64, generator=g) * 0.5)
    c = c.half()
    with torch.no_grad():
        up = F.interpolate(fm, scale_factor=2, mode="bilinear", align_corners=True)
        y = F.conv2d(torch.cat([up, skip], 1), c.weight, None, 1, 1) + c.bias.view(1, -1, 1, 1)
        ref = F.leaky_relu(y, 0.1)
        got = decoder_conv4s(fm, skip, decoder_conv4s_weights(c), 0.1)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    d = (got.float() - ref.float()).abs()
    print(f"decoder conv4s {2 * h}x{2 * w}: max dev {float(d.max()):.3e}, mean {float(d.mean()):.2e} (scale {sc:.2f})")
    assert float(d.max()) <= 2 ** -7 * sc
    assert float(d.mean()) <= 2 ** -12 * sc
    _check_decoder_fp64(got, fm, skip, c, 0.1, "decoder conv4s")


def _check_decoder_fp64(got, fm, skip, c, slope, name, head=None):
    """A decoder kernel against the f64 reference of the same fp16 inputs:
    upsample x2 (align_corners) + cat + 3x3 conv + bias + LeakyReLU (+ the 1x1
    head conv + bias), bounded by the fp16 blend (BLEND x the blended sources'
    largest |fm|, through sum |w|), the f32 accumulation and each fp16
    rounding of the epilogue (tests/fp16_bounds.py)."""
    F = torch.nn.functional
    with torch.no_grad():
        up = F.interpolate(fm.double(), scale_factor=2, mode="bilinear", align_corners=True)
        xin = torch.cat([up, skip.double()], 1)
        cin = xin.shape[1]
        c64 = B.conv64(xin, c.weight, padding=1)
        eb = torch.cat([B.BLEND * B.blend_source_max(fm), torch.zeros_like(skip, dtype=torch.float64)], 1)
        e = B.conv64(eb, c.weight.abs(), padding=1) + B.acc_bound(xin, c.weight, 9 * cin, padding=1)
        e = B.round_step(c64, e)                                    # the conv's fp16 output
        y64 = c64 + c.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)                                    # + bias (fp16 add)
        e = B.leaky_step(y64, e, slope)
        y64 = F.leaky_relu(y64, slope)
        if head is not None:                                        # the tail's 1x1 conv + bias
            w2, b2 = head
            k = w2.shape[1]
            e = B.conv64(e, w2.abs()) + B.acc_bound(y64, w2, k)
            y64 = B.conv64(y64, w2)
            e = B.round_step(y64, e)
            y64 = y64 + b2.double().view(1, -1, 1, 1)
            e = B.round_step(y64, e)
    B.check(got, y64, e, name)


def test_stem_weight_layout():
    """pv_stem_conv_f16's space-to-depth weights (network.stem_weights): the
    4x4 convolution over 2x2-folded pixels they describe equals conv1's 7x7 /
    stride 2 / pad 3 convolution (CPU, f64 emulation of the kernel's sum)."""
    from pvnet_amd.network import stem_weights
    F = torch.nn.functional
    g = torch.Generator().manual_seed(11)
    c = torch.nn.Conv2d(3, 64, 7, 2, 3)
    with torch.no_grad():
        c.weight.copy_(torch.randn(64, 3, 7, 7, generator=g))
    wt, _ = stem_weights(c)
    assert tuple(wt.shape) == (2, 16, 2, 32, 8)
    W2 = wt.double().permute(0, 3, 1, 2, 4).reshape(64, 16, 16)       # [co, tap, s2d channel]
    h, w = 10, 14
    img = torch.randn(1, 3, h, w, generator=g, dtype=torch.float64)
    # s2d pixel (Y, X), channel dy*6 + dx*3 + ci = img[ci][2Y + dy][2X + dx]; 2 pixels of zero border
    s2d = img[0].reshape(3, h // 2, 2, w // 2, 2).permute(1, 3, 2, 4, 0).reshape(h // 2, w // 2, 12)
    s2d = F.pad(torch.cat([s2d, s2d.new_zeros(h // 2, w // 2, 4)], 2), (0, 0, 2, 2, 2, 2))
    got = torch.zeros(64, h // 2, w // 2, dtype=torch.float64)
    for tap in range(16):
        ty, tx = divmod(tap, 4)
        got += torch.einsum("oc,yxc->oyx", W2[:, tap], s2d[ty:ty + h // 2, tx:tx + w // 2])
    ref = F.conv2d(img, c.weight.detach().half().double(), None, 2, 3)[0]
    assert torch.allclose(got, ref, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(480, 640), (38, 70), (34, 126), (18, 62)])
def test_stem_conv_matches_torch(hw, device):
    """pv_stem_conv_f16 (conv1 7x7/2/3 + folded BN + ReLU = x2s, RN:139-142,
    201-203) against MIOpen's fp16 convolution + ATen's bias add and ReLU; then
    the pool-only maxpool against max_pool2d (bit-equal on the same x2s).  Both
    convolutions sum in f32 and round once to fp16 (in other orders): within a
    couple of fp16 roundings of the convolution's scale; ragged tiles (19 x 35
    outputs) included."""
    from pvnet_amd.network import maxpool, stem_conv, stem_weights
    F = torch.nn.functional
    g = torch.Generator().manual_seed(hw[0] + hw[1])
    cl = torch.channels_last
    h, w = hw
    img = torch.randn(2, 3, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    c = torch.nn.Conv2d(3, 64, 7, 2, 3).to(device)
    with torch.no_grad():
        c.weight.copy_(torch.randn(64, 3, 7, 7, generator=g) * 0.1)
        c.bias.copy_(torch.randn(64, generator=g) * 0.5)
    c = c.half()
    with torch.no_grad():
        ref = torch.relu(F.conv2d(img, c.weight, None, 2, 3) + c.bias.view(1, -1, 1, 1))
        got = stem_conv(img, stem_weights(c))
        pool = maxpool(got)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    d = (got.float() - ref.float()).abs()
    print(f"stem conv {h}x{w}: max dev {float(d.max()):.3e}, mean {float(d.mean()):.2e} (scale {sc:.2f})")
    assert float(d.max()) <= 2 ** -7 * sc
    assert float(d.mean()) <= 2 ** -12 * sc
    with torch.no_grad():                     # against an f64 convolution of the same inputs (tests/fp16_bounds.py)
        c64 = B.conv64(img, c.weight, stride=2, padding=3)
        e = B.round_step(c64, B.acc_bound(img, c.weight, 3 * 49, stride=2, padding=3))
        y64 = c64 + c.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)
    B.check(got, torch.relu(y64), e, f"stem conv {h}x{w}")
    assert pool.is_contiguous(memory_format=cl) and torch.equal(pool, F.max_pool2d(got, 3, 2, 1))
    # the fused pass (conv + maxpool, pv_stem_pool_f16): the same x2s, bit for
    # bit, and the pool equal to max_pool2d of it -- tiles of 30 x2s columns and
    # 8 rows, ragged at the right and bottom edges, ranges starting mid-strip
    for nb in (2, 3):
        imgb = img if nb == 2 else torch.cat([img, img[:1].flip(3)]).contiguous(memory_format=cl)
        with torch.no_grad():
            x2, pl = stem_conv(imgb, stem_weights(c), pool=True)
            x2_only = stem_conv(imgb, stem_weights(c))
        torch.cuda.synchronize()
        assert torch.equal(x2, x2_only), f"fused stem x2s {h}x{w} batch {nb}"
        assert pl.is_contiguous(memory_format=cl) and torch.equal(pl, F.max_pool2d(x2_only, 3, 2, 1)), \
            f"fused stem pool {h}x{w} batch {nb}"


def test_conv64_weight_layout():
    """pv_conv64_f16's weight image (network.conv64_weights) follows
    include/pvvote.h's formula W[cout][8q + j][ky][kx] (CPU)."""
    from pvnet_amd.network import conv64_weights
    g = torch.Generator().manual_seed(3)
    c = torch.nn.Conv2d(64, 64, 3, 1, 1)
    with torch.no_grad():
        c.weight.copy_(torch.randn(64, 64, 3, 3, generator=g))
    w = conv64_weights(c)
    W = c.weight.detach().half()
    for tap in range(9):
        for q in range(8):
            assert torch.equal(w[tap, q], W[:, 8 * q: 8 * q + 8, tap // 3, tap % 3])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["relu_120x160", "res_120x160", "none_ragged_13x37", "res_120x160x8"])
def test_conv64_matches_torch(case, device):
    """pv_conv64_f16 (layer1's 64 -> 64 3x3 convolutions with bias, residual
    and ReLU, RN:21-70) against MIOpen's fp16 convolution + ATen's bias /
    residual / ReLU; tolerance as the conv3x3 test; ragged tiles included;
    `x8`: batch 8, more tiles than persistent blocks (the next tile's halo
    prefetched during a tile)."""
    from pvnet_amd.network import conv64, conv64_weights
    F = torch.nn.functional
    kind, hw = case.split("_")[0], case.split("_")[-1]
    dims = [int(v) for v in hw.split("x")]
    h, w, n = dims[0], dims[1], (dims[2] if len(dims) > 2 else 2)
    g = torch.Generator().manual_seed(h * w)
    cl = torch.channels_last
    x = torch.randn(n, 64, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    res = torch.randn(n, 64, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    c = torch.nn.Conv2d(64, 64, 3, 1, 1).to(device)
    with torch.no_grad():
        c.weight.copy_(torch.randn(64, 64, 3, 3, generator=g) / 24)
        c.bias.copy_(torch.randn(64, generator=g) * 0.5)
    c = c.half()
    with torch.no_grad():
        y = F.conv2d(x, c.weight, None, 1, 1) + c.bias.view(1, -1, 1, 1)
        if kind == "res":
            y = y + res
        ref = y if kind == "none" else torch.relu(y)
        got = conv64(x, conv64_weights(c), c.bias, "none" if kind == "none" else "relu",
                     res=res if kind == "res" else None)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=cl)
    sc = float(ref.abs().max())
    d = (got.float() - ref.float()).abs()
    print(f"conv64 {case}: max dev {float(d.max()):.3e}, mean {float(d.mean()):.2e} (scale {sc:.2f})")
    assert float(d.max()) <= 2 ** -8 * sc
    assert float(d.mean()) <= 2 ** -13 * sc
    with torch.no_grad():                     # against an f64 convolution of the same inputs (tests/fp16_bounds.py)
        c64 = B.conv64(x, c.weight, padding=1)
        e = B.round_step(c64, B.acc_bound(x, c.weight, 9 * 64, padding=1))
        y64 = c64 + c.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)
        if kind == "res":
            y64 = y64 + res.double()
            e = B.round_step(y64, e)
        if kind != "none":
            y64 = torch.relu(y64)
    B.check(got, y64, e, f"conv64 {case}")

def test_conv3x3_ex_eligibility():
    """Which convolutions PVNetInference routes to pv_conv3x3_ex_f16 (CPU):
    3x3, stride 1 or 2, padding = dilation, Cin % 64, Cout % 128; and which
    downsamples it sums into conv2 (a 1x1 conv with bias, the folded BN left
    as an Identity)."""
    from torch import nn
    from pvnet_amd.network import PVNet, conv3x3_eligible, downsample_eligible, fold_batchnorm
    assert conv3x3_eligible(nn.Conv2d(64, 128, 3, 2, 1))
    assert conv3x3_eligible(nn.Conv2d(256, 512, 3, 1, 4, 4))
    assert not conv3x3_eligible(nn.Conv2d(64, 128, 3, 3, 1))
    assert not conv3x3_eligible(nn.Conv2d(64, 96, 3, 1, 1))
    assert not conv3x3_eligible(nn.Conv2d(32, 128, 3, 1, 1))
    assert not conv3x3_eligible(nn.Conv2d(64, 128, 3, 1, 2, 1))
    f = fold_batchnorm(PVNet(18, 2).eval())
    r = f.resnet18_8s
    dss = [blk.downsample for layer in (r.layer2, r.layer3, r.layer4) for blk in layer if blk.downsample is not None]
    assert len(dss) == 3 and all(downsample_eligible(d) for d in dss)
    assert not downsample_eligible(None)
    assert not downsample_eligible(nn.Sequential(nn.Conv2d(64, 128, 1, 2, bias=False)))


@pytest.mark.gpu
def test_conv_split_scratch_capture_without_warmup(device):
    """The split-K scratch of pv_conv3x3_ex_f16 and graph capture (advisor,
    rounds 3 and 4): capture a convolution whose last round of tiles is
    split, on a fresh stream with no warm-up, then run the same call eagerly
    on that stream BEFORE any replay, then replay.  The capture takes a
    scratch of its own from the graph's pool and captures the fill of its
    counters; the eager calls make and zero a buffer outside it.  Every
    output is within the fp16 bound of the f64 convolution, and the replay
    and both eager calls are bit-equal (the same split, summed in part
    order)."""
    from pvnet_amd.network import clear_conv_workspaces, conv3x3, conv3x3_weight
    F = torch.nn.functional
    g = torch.Generator().manual_seed(404)
    cl = torch.channels_last
    n, cin, cout, h, w, d = 16, 128, 128, 60, 80, 1
    x = torch.randn(n, cin, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    conv = torch.nn.Conv2d(cin, cout, 3, 1, d, d, bias=True).to(device)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.5)
    conv = conv.half()
    wt = conv3x3_weight(conv)
    clear_conv_workspaces()
    s = torch.cuda.Stream(device=device)
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            got_g = conv3x3(x, wt, conv.bias, d, "relu")
        e1 = conv3x3(x, wt, conv.bias, d, "relu")          # eager, before any replay
        e2 = conv3x3(x, wt, conv.bias, d, "relu")
    s.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(e1, e2)
    assert torch.equal(got_g, e1)
    with torch.no_grad():
        c64 = B.conv64(x, conv.weight, padding=d, dilation=d)
        e = B.round_step(c64, B.acc_bound(x, conv.weight, 9 * cin, padding=d, dilation=d))
        y64 = c64 + conv.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)
        y64 = torch.relu(y64)
    B.check(e1, y64, e, "eager after capture")
    B.check(got_g, y64, e, "captured (replayed)")
    clear_conv_workspaces()


@pytest.mark.gpu
def test_conv_split_scratch_shared_by_two_shapes(device):
    """One stream's split-K scratch serves convolutions of different shapes in
    turn (network._conv_workspace keeps one per stream): shape A (100 split
    tiles on 256 CUs), shape B (30 split tiles), A again.  B's partials must
    not land on A's arrival counters (the counters' region has one size for
    every shape, pvvote.h), so the second A equals the first bit for bit, and
    both are within the fp16 bound of the f64 convolution."""
    from pvnet_amd import _lib
    from pvnet_amd.network import clear_conv_workspaces, conv3x3, conv3x3_weight
    g = torch.Generator().manual_seed(606)
    cl = torch.channels_last
    cin, cout = 128, 128
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=True)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.5)
    conv = conv.to(device).half()
    wt = conv3x3_weight(conv)
    xa = torch.randn(1, cin, 178, 512, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    xb = torch.randn(1, cin, 143, 512, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
    L = _lib.load()
    assert L.pv_conv3x3_workspace_bytes(178 * 512, cout, 18) > 0 and L.pv_conv3x3_workspace_bytes(143 * 512, cout, 18) > 0
    clear_conv_workspaces()
    s = torch.cuda.Stream(device=device)
    with torch.no_grad(), torch.cuda.stream(s):
        a1 = conv3x3(xb, wt, conv.bias, 1, "relu")           # B first: the scratch grows to A's size below
        a1 = conv3x3(xa, wt, conv.bias, 1, "relu")
        conv3x3(xb, wt, conv.bias, 1, "relu")
        a2 = conv3x3(xa, wt, conv.bias, 1, "relu")
    s.synchronize()
    assert torch.equal(a1, a2)
    with torch.no_grad():
        c64 = B.conv64(xa, conv.weight, padding=1)
        e = B.round_step(c64, B.acc_bound(xa, conv.weight, 9 * cin, padding=1))
        y64 = c64 + conv.bias.double().view(1, -1, 1, 1)
        e = B.round_step(y64, e)
        y64 = torch.relu(y64)
    B.check(a2, y64, e, "split scratch shared by two shapes")
    clear_conv_workspaces()
