"""PVNet seg + vector-field network (ResNet-18 at output stride 8, 3-stage
upsampling decoder) on PyTorch-ROCm.

Module tree and state-dict keys are those of ``PVnet``
(lib/networks/model_repository.py:7-79, MR) == ``Resnet18_8s``
(lib/networks/model_repository_orig.py:7-80), so a reference checkpoint's
``['net']`` dict loads with ``strict=True``.  Topology (MR:64-79, RN:116-221):

  conv7x7/2 -> BN -> ReLU (x2s) -> maxpool -> layer1 (x4s) -> layer2/2 (x8s)
  -> layer3 (dilation 2) -> layer4 (dilation 4) -> fc: 3x3 512->256 BN ReLU
  conv8s(cat[xfc, x8s]) -> up x2 -> conv4s(cat[., x4s]) -> up x2
  -> conv2s(cat[., x2s]) -> up x2 -> convraw(cat[., image]) -> 1x1 -> seg 2 + vertex 2K

Upsampling is ``UpsamplingBilinear2d`` (align_corners=True) as in MR:35,43,51.
The module form :class:`PVNet` runs its convolutions through MIOpen; the
inference form :class:`PVNetInference` runs every fp16 convolution (with its
epilogue) as one of this repository's HIP matrix-core kernels
(``pvnet_amd/csrc/pvconv.hip``) and, in f32, MIOpen + HIP epilogue passes.
``channels_last`` and fp16 are the MI355X knobs (the reference's fp16 precedent:
python-only-xin/pvnet-master/tools/train_linemod.py:514).  No weights ship with
the reference (README.md:101 points to a download), so the default init is the
reference's own (RN:156-163: He-normal convs, BN weight 1 / bias 0).
"""
from __future__ import annotations

import math
import threading

import torch
import torch.nn.functional as F
from torch import nn


def _conv3x3(cin, cout, stride=1, dilation=1):
    # RN:21-38: padding keeps the spatial size for any dilation
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=dilation, dilation=dilation, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = _conv3x3(cin, cout, stride, dilation)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(cout, cout, dilation=dilation)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + idt)


class ResNet18OS8(nn.Module):
    """ResNet-18 whose layer3/layer4 trade stride for dilation (RN:167-198).
    Keeps the reference's unused ``avgpool`` attribute so the module tree (and
    therefore the state-dict keys) match."""

    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        # (planes, blocks, stride, dilation) after the output-stride rule: OS 8 is
        # reached after layer2, so layer3/4 keep stride 1 with dilation 2/4.
        self.layer1 = self._layer(64, 2, 1, 1, False)
        self.layer2 = self._layer(128, 2, 2, 1, True)
        self.layer3 = self._layer(256, 2, 1, 2, True)
        self.layer4 = self._layer(512, 2, 1, 4, True)
        self.avgpool = nn.AvgPool2d(7, padding=3, stride=1)
        self.fc = nn.Identity()   # replaced by PVNet (MR:22-26)

    def _layer(self, planes, blocks, stride, dilation, down):
        ds = None
        if down:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride=stride, bias=False), nn.BatchNorm2d(planes))
        mods = [BasicBlock(self.inplanes, planes, stride, ds, dilation)]
        self.inplanes = planes
        mods += [BasicBlock(planes, planes, dilation=dilation) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        x2s = self.relu(self.bn1(self.conv1(x)))
        x4s = self.layer1(self.maxpool(x2s))
        x8s = self.layer2(x4s)
        x16s = self.layer3(x8s)
        x32s = self.layer4(x16s)
        return x2s, x4s, x8s, x16s, x32s, self.fc(x32s)


def _cbl(cin, cout, leaky=True):
    return nn.Sequential(nn.Conv2d(cin, cout, 3, 1, 1, bias=False), nn.BatchNorm2d(cout),
                         nn.LeakyReLU(0.1, True) if leaky else nn.ReLU(True))


class PVNet(nn.Module):
    """``PVnet(ver_dim, seg_dim)`` of MR:7-79 (alias :data:`Resnet18_8s`)."""

    def __init__(self, ver_dim=18, seg_dim=2, fcdim=256, s8dim=128, s4dim=64, s2dim=32, raw_dim=32):
        super().__init__()
        self.ver_dim, self.seg_dim = ver_dim, seg_dim
        r = ResNet18OS8()
        r.fc = _cbl(512, fcdim, leaky=False)
        self.resnet18_8s = r
        self.conv8s = _cbl(128 + fcdim, s8dim)
        self.up8sto4s = nn.UpsamplingBilinear2d(scale_factor=2)
        self.conv4s = _cbl(64 + s8dim, s4dim)
        self.up4sto2s = nn.UpsamplingBilinear2d(scale_factor=2)
        self.conv2s = _cbl(64 + s4dim, s2dim)
        self.up2storaw = nn.UpsamplingBilinear2d(scale_factor=2)
        self.convraw = nn.Sequential(nn.Conv2d(3 + s2dim, raw_dim, 3, 1, 1, bias=False), nn.BatchNorm2d(raw_dim),
                                     nn.LeakyReLU(0.1, True), nn.Conv2d(raw_dim, seg_dim + ver_dim, 1, 1))
        self.reset_parameters()

    def reset_parameters(self):
        """RN:156-163 for every conv / BN (the decoder is built after the
        backbone in MR, so torch's default init applies there; we use the
        backbone rule throughout -- no reference weights exist offline)."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def forward(self, x):
        x2s, x4s, x8s, _, _, xfc = self.resnet18_8s(x)
        fm = self.up8sto4s(self.conv8s(torch.cat([xfc, x8s], 1)))
        fm = self.up4sto2s(self.conv4s(torch.cat([fm, x4s], 1)))
        fm = self.up2storaw(self.conv2s(torch.cat([fm, x2s], 1)))
        x = self.convraw(torch.cat([fm, x], 1))
        return x[:, :self.seg_dim], x[:, self.seg_dim:]


Resnet18_8s = PVNet
PVnet = PVNet


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    """conv followed by eval-mode bn as one convolution with a bias: per output
    channel k, w'_k = w_k g_k and b'_k = beta_k + (b_k - mean_k) g_k with
    g_k = gamma_k / sqrt(var_k + eps) (folded in fp64, stored in conv's dtype)."""
    g = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    b0 = conv.bias.double() if conv.bias is not None else torch.zeros_like(g)
    out = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                    conv.dilation, conv.groups, bias=True, padding_mode=conv.padding_mode,
                    device=conv.weight.device, dtype=conv.weight.dtype)
    out.weight.copy_((conv.weight.double() * g.view(-1, 1, 1, 1)).to(conv.weight.dtype))
    out.bias.copy_((bn.bias.double() + (b0 - bn.running_mean.double()) * g).to(conv.weight.dtype))
    return out


@torch.no_grad()
def fold_batchnorm(net: nn.Module) -> nn.Module:
    """Inference copy of a PVNet with every BatchNorm2d folded into the
    convolution before it (the BN becomes ``nn.Identity``): 25 fewer
    normalisation passes over the activations per forward, the same function
    up to rounding.  Load a checkpoint into :class:`PVNet` first (the folded
    copy's state-dict keys differ); the copy is eval-only."""
    import copy
    net = copy.deepcopy(net).eval()
    for m in list(net.modules()):
        if isinstance(m, BasicBlock):
            m.conv1, m.bn1 = _fold(m.conv1, m.bn1), nn.Identity()
            m.conv2, m.bn2 = _fold(m.conv2, m.bn2), nn.Identity()
        elif isinstance(m, ResNet18OS8):
            m.conv1, m.bn1 = _fold(m.conv1, m.bn1), nn.Identity()
        elif isinstance(m, nn.Sequential):
            for i in range(len(m) - 1):
                if isinstance(m[i], nn.Conv2d) and isinstance(m[i + 1], nn.BatchNorm2d):
                    m[i], m[i + 1] = _fold(m[i], m[i + 1]), nn.Identity()
    assert not any(isinstance(m, nn.BatchNorm2d) for m in net.modules()), "a BatchNorm2d was left unfolded"
    return net


def upsample2x_cat(fm: torch.Tensor, skip: torch.Tensor | None, cpad: int) -> torch.Tensor:
    """``torch.cat([UpsamplingBilinear2d(2)(fm), skip], 1)`` zero-padded to
    ``cpad`` channels, for channels-last fp16 / f32 device tensors, in one HIP
    pass (``pv_upsample2x_cat_f16`` / ``_f32``, pvnet_amd/csrc/pvdecoder.hip)."""
    from pvnet_amd import _lib
    n, c1, h, w = fm.shape
    c2 = 0 if skip is None else skip.shape[1]
    cl = torch.channels_last
    fn = {torch.float16: "pv_upsample2x_cat_f16", torch.float32: "pv_upsample2x_cat_f32"}.get(fm.dtype)
    if fn is None or not fm.is_cuda or not fm.is_contiguous(memory_format=cl):
        raise RuntimeError("upsample2x_cat: fm must be a channels_last float16 / float32 CUDA tensor")
    if skip is not None and (skip.dtype != fm.dtype or not skip.is_contiguous(memory_format=cl)
                             or tuple(skip.shape) != (n, c2, 2 * h, 2 * w)):
        raise RuntimeError("upsample2x_cat: skip must be channels_last [n, c2, 2h, 2w] of fm's dtype")
    out = torch.empty((n, cpad, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
    stream = torch.cuda.current_stream(fm.device).cuda_stream
    _lib.check(getattr(_lib.load(), fn)(fm.data_ptr(), None if skip is None else skip.data_ptr(),
                                        out.data_ptr(), n, h, w, c1, c2, cpad, stream), fn)
    return out


def _dev_call(fn16, fn32, t: torch.Tensor, *args):
    from pvnet_amd import _lib
    fn = {torch.float16: fn16, torch.float32: fn32}.get(t.dtype)
    if fn is None or not t.is_cuda:
        raise RuntimeError(f"{fn16[:-4]}: a float16 / float32 CUDA tensor is required")
    _lib.check(getattr(_lib.load(), fn)(*args, torch.cuda.current_stream(t.device).cuda_stream), fn)


_ACT = {"none": 0, "relu": 1, "leaky": 2}


def conv_epilogue(y: torch.Tensor, bias: torch.Tensor, act: str = "relu", res: torch.Tensor | None = None,
                  rbias: torch.Tensor | None = None, skip: torch.Tensor | None = None,
                  slope: float = 0.1) -> torch.Tensor:
    """``act(y + bias [+ (res + rbias)])`` over a channels-last conv output in
    one HIP pass (``pv_conv_epilogue_f16/_f32``), in place -- or, with
    ``skip``, written beside it as ``torch.cat([.., skip], 1)`` into a new
    tensor.  ATen's roundings of the unfused bias add / residual add /
    activation (RN:41-70, MR:22-58)."""
    n, c1, h, w = y.shape
    cl = torch.channels_last
    for t in (y, res, skip):
        if t is not None and not t.is_contiguous(memory_format=cl):
            raise RuntimeError("conv_epilogue: channels_last maps required")
    c2 = 0 if skip is None else skip.shape[1]
    out = y if skip is None else torch.empty((n, c1 + c2, h, w), dtype=y.dtype, device=y.device, memory_format=cl)
    _dev_call("pv_conv_epilogue_f16", "pv_conv_epilogue_f32", y, y.data_ptr(), bias.data_ptr(),
              None if res is None else res.data_ptr(), None if rbias is None else rbias.data_ptr(),
              None if skip is None else skip.data_ptr(), out.data_ptr(), n * h * w, c1, c2, _ACT[act], float(slope))
    return out


def head(y: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, slope: float = 0.1) -> torch.Tensor:
    """convraw's tail (MR:53-58) after its 3x3 convolution: bias + LeakyReLU +
    the 1x1 convolution with its bias, one HIP pass (``pv_head_f16/_f32``).
    y [n, 32, h, w] channels_last; b1 / w2 [cout, 32] / b2 float32 device."""
    n, cin, h, w = y.shape
    cout = w2.shape[0]
    if not y.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("head: channels_last input required")
    out = torch.empty((n, cout, h, w), dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
    _dev_call("pv_head_f16", "pv_head_f32", y, y.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
              out.data_ptr(), n * h * w, cin, cout, float(slope))
    return out


def relu_maxpool(y: torch.Tensor, bias: torch.Tensor):
    """The stem's tail (RN:201-204) after conv1, BN folded: x2s = relu(y +
    bias) and maxpool3x3/2/1(x2s) from one HIP pass (``pv_relu_maxpool_f16 /
    _f32``), both bit-equal to ATen's ops.  y [n, c, h, w] channels_last."""
    n, c, h, w = y.shape
    cl = torch.channels_last
    if not y.is_contiguous(memory_format=cl):
        raise RuntimeError("relu_maxpool: channels_last input required")
    x2s = torch.empty_like(y, memory_format=cl)
    pool = torch.empty((n, c, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=y.dtype, device=y.device, memory_format=cl)
    _dev_call("pv_relu_maxpool_f16", "pv_relu_maxpool_f32", y, y.data_ptr(), bias.data_ptr(), x2s.data_ptr(),
              pool.data_ptr(), n, h, w, c)
    return x2s, pool


def maxpool(x2s: torch.Tensor):
    """maxpool 3x3 / 2 / 1 (RN:204) of a channels-last map in one HIP pass
    (``pv_relu_maxpool_f16 / _f32``'s pool-only form): bit-equal to ATen's."""
    n, c, h, w = x2s.shape
    cl = torch.channels_last
    if not x2s.is_contiguous(memory_format=cl):
        raise RuntimeError("maxpool: channels_last input required")
    pool = torch.empty((n, c, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=x2s.dtype, device=x2s.device,
                       memory_format=cl)
    _dev_call("pv_relu_maxpool_f16", "pv_relu_maxpool_f32", x2s, x2s.data_ptr(), None, None, pool.data_ptr(),
              n, h, w, c)
    return pool


def stem_eligible(c: nn.Conv2d) -> bool:
    """conv1 as ``pv_stem_conv_f16`` takes it: 7x7, stride 2, padding 3, 3 -> 64."""
    return (c.kernel_size == (7, 7) and c.stride == (2, 2) and c.padding == (3, 3) and c.dilation == (1, 1)
            and c.groups == 1 and c.in_channels == 3 and c.out_channels == 64)


def stem_weights(c: nn.Conv2d):
    """conv1's weights (BN folded) in ``pv_stem_conv_f16``'s space-to-depth
    layout and its bias, fp16: tap (ty, tx) of the 4x4 convolution over 2x2-
    folded pixels, channel dy*6 + dx*3 + ci = W[ci][2ty+dy-1][2tx+dx-1] (zero
    outside the 7x7), as the lanes' A fragments [2][16][2][32][8]."""
    if not stem_eligible(c):
        raise RuntimeError("stem_weights: conv1 must be a 7x7 / 2 / pad 3, 3 -> 64 convolution")
    w = c.weight.detach().float()                                   # [64, 3, 7, 7]
    w8 = torch.zeros(64, 3, 8, 8, dtype=w.dtype, device=w.device)
    w8[:, :, 1:, 1:] = w                                            # index 2t + d = k + 1
    w2 = w8.reshape(64, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1)    # [co, ty, tx, dy, dx, ci]
    w2 = torch.cat([w2.reshape(64, 16, 12), w2.new_zeros(64, 16, 4)], 2)   # [co, tap, 16]
    w2 = w2.reshape(2, 32, 16, 2, 8).permute(0, 2, 3, 1, 4)        # [m, tap, h, n, 8]
    b = c.bias.detach().half().contiguous() if c.bias is not None else torch.zeros(64, dtype=torch.half,
                                                                                    device=w.device)
    return w2.contiguous().half(), b


def stem_conv(img: torch.Tensor, weights, pool: bool = False):
    """relu(conv1(img) + b) (RN:139-142, 201-203; BN folded) as one fp16
    matrix-core pass (``pv_stem_conv_f16``): img [n, 3, h, w] channels_last
    float16 CUDA, h and w even; ``weights`` from :func:`stem_weights`.
    Returns x2s [n, 64, h/2, w/2] channels_last; with ``pool`` also
    maxpool 3x3 / 2 / 1 of it (RN:204) from the same pass
    (``pv_stem_pool_f16``): (x2s, pool)."""
    n, c, h, w = img.shape
    if img.dtype != torch.float16 or not img.is_cuda or c != 3:
        raise RuntimeError("stem_conv: a [n, 3, h, w] float16 CUDA image required")
    if h % 2 or w % 2 or not img.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("stem_conv: channels_last, even h and w required")
    wt, b = weights
    out = torch.empty((n, 64, h // 2, w // 2), dtype=img.dtype, device=img.device,
                      memory_format=torch.channels_last)
    if not pool:
        _dev_call("pv_stem_conv_f16", None, img, img.data_ptr(), wt.data_ptr(), b.data_ptr(), out.data_ptr(), n, h, w)
        return out
    ho, wo = h // 2, w // 2
    pl = torch.empty((n, 64, (ho - 1) // 2 + 1, (wo - 1) // 2 + 1), dtype=img.dtype, device=img.device,
                     memory_format=torch.channels_last)
    _dev_call("pv_stem_pool_f16", None, img, img.data_ptr(), wt.data_ptr(), b.data_ptr(), out.data_ptr(),
              pl.data_ptr(), n, h, w)
    return out, pl


def conv64_eligible(c: nn.Conv2d) -> bool:
    """The convolutions ``pv_conv64_f16`` takes: layer1's 3x3 / stride 1 / pad
    1, 64 -> 64."""
    return (c.kernel_size == (3, 3) and c.stride == (1, 1) and c.padding == (1, 1) and c.dilation == (1, 1)
            and c.groups == 1 and c.in_channels == 64 and c.out_channels == 64)


def conv64_weights(c: nn.Conv2d) -> torch.Tensor:
    """A 64 -> 64 3x3 weight (BN folded) as ``pv_conv64_f16`` reads it: [9 taps
    (ky, kx)][8 octets q][64 couts][8] fp16 = W[cout][8q + j][ky][kx]."""
    if not conv64_eligible(c):
        raise RuntimeError("conv64_weights: a 3x3 / stride 1 / pad 1, 64 -> 64 convolution required")
    w = c.weight.detach().float().reshape(64, 8, 8, 3, 3).permute(3, 4, 1, 0, 2)   # [ky, kx, q, cout, j]
    return w.reshape(9, 8, 64, 8).contiguous().half()


def conv64(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, act: str = "relu",
           res: torch.Tensor | None = None) -> torch.Tensor:
    """``act(conv(x) + bias (+ res))`` for layer1's 64 -> 64 3x3 convolutions
    in one fp16 matrix-core pass (``pv_conv64_f16``): x / res [n, 64, h, w]
    channels_last float16 CUDA, ``w`` from :func:`conv64_weights`."""
    n, c, h, wd = x.shape
    cl = torch.channels_last
    if x.dtype != torch.float16 or not x.is_cuda or c != 64 or not x.is_contiguous(memory_format=cl):
        raise RuntimeError("conv64: a [n, 64, h, w] channels_last float16 CUDA map required")
    if res is not None and (tuple(res.shape) != tuple(x.shape) or not res.is_contiguous(memory_format=cl)):
        raise RuntimeError("conv64: residual [n, 64, h, w] channels_last required")
    if act not in ("none", "relu"):
        raise RuntimeError("conv64: act none or relu")
    out = torch.empty_like(x, memory_format=cl)
    _dev_call("pv_conv64_f16", None, x, x.data_ptr(), w.data_ptr(), bias.data_ptr(),
              None if res is None else res.data_ptr(), out.data_ptr(), n, h, wd, _ACT[act])
    return out


def conv3x3_eligible(c: nn.Conv2d) -> bool:
    """The convolutions ``pv_conv3x3_ex_f16`` takes: 3x3, stride 1 or 2,
    padding = dilation, no groups, Cin a multiple of 64, Cout of 128 (layer2
    -- its stride-2 first convolution included --, layer3, layer4, fc,
    conv8s)."""
    return (c.kernel_size == (3, 3) and c.stride[0] == c.stride[1] and c.stride[0] in (1, 2) and c.groups == 1
            and c.padding == c.dilation and c.dilation[0] == c.dilation[1] and c.in_channels % 64 == 0
            and c.out_channels % 128 == 0)


def downsample_eligible(ds) -> bool:
    """A BasicBlock downsample ``pv_conv3x3_ex_f16`` sums into conv2's
    accumulator (PV_CONV_X2_1X1): one 1x1 convolution (BN folded), no
    padding, Cin a multiple of 64."""
    if ds is None or not isinstance(ds[0], nn.Conv2d) or not all(isinstance(m, nn.Identity) for m in ds[1:]):
        return False                  # (fold_batchnorm leaves the folded BN as an Identity)
    d = ds[0]
    return (d.kernel_size == (1, 1) and d.padding == (0, 0) and d.groups == 1 and d.stride[0] == d.stride[1]
            and d.in_channels % 64 == 0 and d.bias is not None)


def conv3x3(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, dil: int, act: str = "relu",
            res: torch.Tensor | None = None, rbias: torch.Tensor | None = None, slope: float = 0.1,
            extra: int = 0) -> torch.Tensor:
    """A wide 3x3 convolution and its epilogue, ``act(conv(x) + bias (+ (res
    + rbias)))``, in one matrix-core pass (``pv_conv3x3_f16``): x [n, cin, h,
    w] channels_last float16, w [cout, 3, 3, cin] contiguous (see
    :func:`conv3x3_weight`), bias / rbias [cout] float16.  ``extra`` > 0:
    the result is [n, cout + extra, h, w] with channels cout.. left for the
    caller (the torch.cat after fc)."""
    n, cin, h, wd = x.shape
    cout = w.shape[0]
    cl = torch.channels_last
    if x.dtype != torch.float16 or not x.is_cuda or not x.is_contiguous(memory_format=cl):
        raise RuntimeError("conv3x3: a channels_last float16 CUDA input is required")
    if tuple(w.shape) != (cout, 3, 3, cin) or not w.is_contiguous() or w.dtype != torch.float16:
        raise RuntimeError("conv3x3: weight [cout, 3, 3, cin] contiguous float16 required")
    if res is not None and (tuple(res.shape) != (n, cout, h, wd) or not res.is_contiguous(memory_format=cl)):
        raise RuntimeError("conv3x3: residual [n, cout, h, w] channels_last required")
    out = torch.empty((n, cout + extra, h, wd), dtype=x.dtype, device=x.device, memory_format=cl)
    ws, wsb = _conv_workspace(x, n * h * wd, cout, 9 * cin // 64)
    _dev_call("pv_conv3x3_ex_f16", None, x, x.data_ptr(), h, wd, 1, None, 0, 0, 0, 0, 0, w.data_ptr(),
              bias.data_ptr(), None if res is None else res.data_ptr(), None if rbias is None else rbias.data_ptr(),
              out.data_ptr(), cout + extra, n, h, wd, cin, cout, int(dil), _ACT[act], float(slope), ws, wsb)
    return out


_CONV_WS: dict = {}         # eager calls: (device, stream) -> [buffers]
_CAPTURE_WS: dict = {}      # inside a capture: (device, stream, capture id) -> the graph's own buffer
_CONV_WS_LOCK = threading.Lock()     # per-GPU threads (DataParallel-style callers) share the tables
_CAPTURE_WS_BYTES = (64 << 20) + 4096


def clear_conv_workspaces() -> None:
    """Drop every eager split-K scratch buffer (no captured graph that used
    one may be replayed afterwards; graph-owned scratch lives in the graphs'
    own memory pools)."""
    with _CONV_WS_LOCK:
        _CONV_WS.clear()
        _CAPTURE_WS.clear()

CONV_SPLIT = True          # the split-K last round (A/B hook for tools/backbone_ab2.py; no environment switch)
TAIL_SPLIT = True          # seg / ver as two dense maps from the fused tail (A/B hook for tools/e2e_vote_probe.py)


def _conv_workspace(x: torch.Tensor, pixels: int, cout: int, ksteps: int):
    """The split-K scratch of pv_conv3x3_ex_f16 (its last partial round of
    tiles; arrival counters that must start at zero, then f32 partials).

    Eager calls: one buffer per (device, stream), since calls on one stream
    run in order; zero-filled when made, grown to the largest need and kept
    (every call leaves its counters at zero again).

    Inside a graph capture: a buffer of the capture's own, per (stream,
    capture id) -- taken from the graph's private memory pool, its counters
    zeroed by a fill captured before the capture's first convolution on that
    stream (so every replay starts from zero).  Graphs captured on one shared
    stream therefore never share counters and can replay concurrently.
    (pointer, bytes) or (None, 0)."""
    from pvnet_amd import _lib
    from pvnet_amd import streams
    L = _lib.load()
    need = int(L.pv_conv3x3_workspace_bytes(pixels, cout, ksteps))
    if need <= 0 or not CONV_SPLIT:
        return None, 0
    stream = torch.cuda.current_stream(x.device)
    if torch.cuda.is_current_stream_capturing():
        cid = streams.capture_id(stream)
        key = (x.device, stream.cuda_stream, cid)
        with _CONV_WS_LOCK:
            for k in [k for k in _CAPTURE_WS if k[2] != cid]:
                del _CAPTURE_WS[k]      # an earlier capture's: its graph's pool keeps the memory
            buf = _CAPTURE_WS.get(key)
            if buf is None or buf.numel() < need:
                # sized for any split of the capture's later convolutions too (at
                # most one split tile per CU, 4 parts of 256 x 256 f32 partials:
                # 64 MiB), so the capture takes one counter fill, not one per size
                buf = torch.empty(max(need, _CAPTURE_WS_BYTES), dtype=torch.uint8, device=x.device)
                nc = int(L.pv_conv3x3_workspace_counter_bytes(pixels, cout, ksteps))   # 4 KiB for every shape
                buf[:nc].zero_()        # captured: runs at every replay, before this call's kernel
                _CAPTURE_WS[key] = buf
            return buf.data_ptr(), buf.numel()
    key = (x.device, stream.cuda_stream)
    with _CONV_WS_LOCK:
        bufs = _CONV_WS.setdefault(key, [])
        if not bufs or bufs[-1].numel() < need:
            # a smaller buffer is kept alive too: a graph captured with it before still uses it
            bufs.append(torch.zeros(need, dtype=torch.uint8, device=x.device))   # zeroed once (pvvote.h)
        return bufs[-1].data_ptr(), bufs[-1].numel()


def conv3x3_weight(c: nn.Conv2d, ds: nn.Conv2d | None = None) -> torch.Tensor:
    """c's weight as pv_conv3x3_f16 reads it: [cout, 3, 3, cin], fp16, contiguous;
    with ``ds`` (a 1x1 downsample) [cout, 9 cin + cin_ds]: the 1x1 weights
    appended to each output channel's row (pv_conv3x3_ex_f16, PV_CONV_X2_1X1)."""
    w = c.weight.detach().permute(0, 2, 3, 1).contiguous().half()
    if ds is None:
        return w
    wd = ds.weight.detach().reshape(ds.out_channels, ds.in_channels).half()
    return torch.cat([w.reshape(c.out_channels, -1), wd], 1).contiguous()


def conv3x3_ex(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, dil: int, stride: int = 1, act: str = "relu",
               x2: torch.Tensor | None = None, mode2: str = "none", s2: int = 1, rbias: torch.Tensor | None = None,
               res: torch.Tensor | None = None, slope: float = 0.1) -> torch.Tensor:
    """``pv_conv3x3_ex_f16``: a 3x3 convolution of x at ``stride`` (padding =
    dilation) and its epilogue, with an optional second input: ``mode2``
    "cat" -- the convolution runs over ``torch.cat([x, x2], 1)`` (w [cout, 3,
    3, cin + cin2]); "1x1" -- a 1x1 convolution of x2 at stride ``s2`` is
    summed into the same accumulator (w [cout, 9 cin + cin2],
    :func:`conv3x3_weight` with ``ds``), its bias ``rbias`` added after
    ``bias``.  channels_last float16 CUDA maps."""
    n, cin, hin, win = x.shape
    cout = w.shape[0]
    cl = torch.channels_last
    h, wd = (hin - 1) // stride + 1, (win - 1) // stride + 1
    m2 = {"none": 0, "cat": 1, "1x1": 2}[mode2]
    for t in (x, x2, res):
        if t is not None and (t.dtype != torch.float16 or not t.is_cuda or not t.is_contiguous(memory_format=cl)):
            raise RuntimeError("conv3x3_ex: channels_last float16 CUDA maps required")
    cin2, h2, w2 = (0, 0, 0) if x2 is None else (x2.shape[1], x2.shape[2], x2.shape[3])
    if (m2 == 0) != (x2 is None) or (m2 == 1 and (h2, w2) != (hin, win)) or x2 is not None and x2.shape[0] != n:
        raise RuntimeError("conv3x3_ex: second input does not match mode2")
    k = 9 * (cin + (cin2 if m2 == 1 else 0)) + (cin2 if m2 == 2 else 0)
    if w.dtype != torch.float16 or not w.is_contiguous() or w.numel() != cout * k:
        raise RuntimeError("conv3x3_ex: weight [cout, K] contiguous float16 required")
    out = torch.empty((n, cout, h, wd), dtype=x.dtype, device=x.device, memory_format=cl)
    ws, wsb = _conv_workspace(x, n * h * wd, cout, k // 64)
    _dev_call("pv_conv3x3_ex_f16", None, x, x.data_ptr(), hin, win, int(stride),
              None if x2 is None else x2.data_ptr(), m2, cin2, h2, w2, int(s2), w.data_ptr(), bias.data_ptr(),
              None if res is None else res.data_ptr(), None if rbias is None else rbias.data_ptr(), out.data_ptr(),
              cout, n, h, wd, cin, cout, int(dil), _ACT[act], float(slope), ws, wsb)
    return out


def decoder_conv2s_weights(c: nn.Conv2d):
    """conv2s's 3x3 weights (BN folded, 128 -> 32) in ``pv_decoder_conv2s_f16``'s
    layout [2][9][8][32][8] fp16 and its bias (fp16)."""
    if c.kernel_size != (3, 3) or c.in_channels != 128 or c.out_channels != 32 or c.padding != (1, 1):
        raise RuntimeError("decoder_conv2s: conv2s must be a 3x3, 128 -> 32, padding-1 convolution")
    w = c.weight.detach().float()                                   # [32, 128, 3, 3]
    w = w.reshape(32, 2, 8, 8, 3, 3).permute(1, 4, 5, 2, 0, 3)      # [part, ky, kx, q, cout, j]
    return w.reshape(2, 9, 8, 32, 8).contiguous().half(), c.bias.detach().half().contiguous()


def decoder_conv2s(fm: torch.Tensor, skip: torch.Tensor, weights, slope: float = 0.1) -> torch.Tensor:
    """up4sto2s + torch.cat([fm, x2s], 1) + conv2s (MR:43-51) in one fp16
    matrix-core pass (``pv_decoder_conv2s_f16``): fm [n, 64, h, w] and skip
    [n, 64, 2h, 2w] channels_last float16 CUDA; ``weights`` from
    :func:`decoder_conv2s_weights`.  Returns [n, 32, 2h, 2w] channels_last."""
    n, c, h, w = fm.shape
    cl = torch.channels_last
    if fm.dtype != torch.float16 or skip.dtype != torch.float16 or not fm.is_cuda:
        raise RuntimeError("decoder_conv2s: float16 CUDA maps required")
    if c != 64 or tuple(skip.shape) != (n, 64, 2 * h, 2 * w):
        raise RuntimeError("decoder_conv2s: fm [n, 64, h, w] and skip [n, 64, 2h, 2w] required")
    if not fm.is_contiguous(memory_format=cl) or not skip.is_contiguous(memory_format=cl):
        raise RuntimeError("decoder_conv2s: channels_last maps required")
    wt, b = weights
    out = torch.empty((n, 32, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
    _dev_call("pv_decoder_conv2s_f16", None, fm, fm.data_ptr(), skip.data_ptr(), wt.data_ptr(), b.data_ptr(),
              out.data_ptr(), n, h, w, float(slope))
    return out


def decoder_conv4s_weights(c: nn.Conv2d):
    """conv4s's 3x3 weights (BN folded, 192 -> 64) in ``pv_decoder_conv4s_f16``'s
    layout [3][9][8][2][32][8] fp16 and its bias (fp16)."""
    if c.kernel_size != (3, 3) or c.in_channels != 192 or c.out_channels != 64 or c.padding != (1, 1):
        raise RuntimeError("decoder_conv4s: conv4s must be a 3x3, 192 -> 64, padding-1 convolution")
    w = c.weight.detach().float()                                            # [64, 192, 3, 3]
    w = w.reshape(2, 32, 3, 8, 8, 3, 3).permute(2, 5, 6, 3, 0, 1, 4)       # [p, ky, kx, q, m, c, j]
    return w.reshape(3, 9, 8, 2, 32, 8).contiguous().half(), c.bias.detach().half().contiguous()


def decoder_conv4s(fm: torch.Tensor, skip: torch.Tensor, weights, slope: float = 0.1) -> torch.Tensor:
    """up8sto4s + torch.cat([fm, x4s], 1) + conv4s (MR:35-43) in one fp16
    matrix-core pass (``pv_decoder_conv4s_f16``): fm [n, 128, h, w] and skip
    [n, 64, 2h, 2w] channels_last float16 CUDA.  Returns [n, 64, 2h, 2w]."""
    n, c, h, w = fm.shape
    cl = torch.channels_last
    if fm.dtype != torch.float16 or skip.dtype != torch.float16 or not fm.is_cuda:
        raise RuntimeError("decoder_conv4s: float16 CUDA maps required")
    if c != 128 or tuple(skip.shape) != (n, 64, 2 * h, 2 * w):
        raise RuntimeError("decoder_conv4s: fm [n, 128, h, w] and skip [n, 64, 2h, 2w] required")
    if not fm.is_contiguous(memory_format=cl) or not skip.is_contiguous(memory_format=cl):
        raise RuntimeError("decoder_conv4s: channels_last maps required")
    wt, b = weights
    out = torch.empty((n, 64, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
    _dev_call("pv_decoder_conv4s_f16", None, fm, fm.data_ptr(), skip.data_ptr(), wt.data_ptr(), b.data_ptr(),
              out.data_ptr(), n, h, w, float(slope))
    return out


def decoder_tail_weights(c0: nn.Conv2d, c1: nn.Conv2d, cin: int = 35):
    """convraw's weights (MR:53-58, BN folded into ``c0``) laid out for
    ``pv_decoder_tail_f16`` (include/pvvote.h): w1 [32][368] fp16 with
    k = (3 ky + kx) * 40 + input channel, b1 f32, w2 in the matrix core
    accumulator's row order [cout/32][2][32][16] fp16, b2 f32."""
    co = c0.out_channels
    if co != 32 or c0.kernel_size != (3, 3) or c1.in_channels != 32 or c1.out_channels not in (20, 44):
        raise RuntimeError("decoder_tail: convraw must be 3x3 conv to 32 channels and 1x1 conv to 20 / 44")
    dev = c0.weight.device
    w = torch.zeros(co, 3, 3, 40, dtype=torch.float32, device=dev)
    w[..., :cin] = c0.weight.detach().float()[:, :cin].permute(0, 2, 3, 1)
    w1 = torch.zeros(co, 368, dtype=torch.float32, device=dev)
    w1[:, :360] = w.reshape(co, 360)
    cout = c1.out_channels
    mt = (cout + 31) // 32
    W2 = torch.zeros(mt * 32, 32, dtype=torch.float32, device=dev)
    W2[:cout] = c1.weight.detach().float().reshape(cout, 32)
    s, h, j = torch.meshgrid(torch.arange(2), torch.arange(2), torch.arange(8), indexing="ij")
    rows = ((j & 3) + 8 * (j >> 2) + 16 * s + 4 * h).to(dev)              # [s][h][j]
    w2 = W2.reshape(mt, 32, 32)[:, :, rows]                               # [t][m][s][h][j]
    w2 = w2.permute(0, 2, 1, 3, 4).reshape(mt, 2, 32, 16)
    return (w1.half().contiguous(), c0.bias.detach().float().contiguous(), w2.half().contiguous(),
            c1.bias.detach().float().contiguous())


def decoder_tail(fm: torch.Tensor, img: torch.Tensor, weights, slope: float = 0.1, split: bool = False):
    """up2storaw + torch.cat([fm, x], 1) + convraw (MR:75-79) in one fp16
    matrix-core pass (``pv_decoder_tail_f16``): fm [n, 32, h, w] and img
    [n, 3, 2h, 2w] channels_last float16 CUDA; ``weights`` from
    :func:`decoder_tail_weights`.  Returns [n, cout, 2h, 2w] channels_last;
    with ``split`` (``pv_decoder_tail_split_f16``) the pair (seg [n, 2, 2h,
    2w], ver [n, cout - 2, 2h, 2w]) as MR:79 slices them, each its own dense
    channels_last map -- the voting layer's argmax then reads 4 bytes per
    pixel, not the cache lines of the whole cout-channel record."""
    n, c, h, w = fm.shape
    cl = torch.channels_last
    if fm.dtype != torch.float16 or img.dtype != torch.float16 or not fm.is_cuda:
        raise RuntimeError("decoder_tail: float16 CUDA maps required")
    if c != 32 or tuple(img.shape) != (n, 3, 2 * h, 2 * w):
        raise RuntimeError("decoder_tail: fm [n, 32, h, w] and img [n, 3, 2h, 2w] required")
    if not fm.is_contiguous(memory_format=cl) or not img.is_contiguous(memory_format=cl):
        raise RuntimeError("decoder_tail: channels_last maps required")
    w1, b1, w2, b2 = weights
    cout = b2.numel()
    if split:
        seg = torch.empty((n, 2, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
        ver = torch.empty((n, cout - 2, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
        _dev_call("pv_decoder_tail_split_f16", None, fm, fm.data_ptr(), img.data_ptr(), w1.data_ptr(),
                  b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), seg.data_ptr(), ver.data_ptr(), n, h, w, cout,
                  float(slope))
        return seg, ver
    out = torch.empty((n, cout, 2 * h, 2 * w), dtype=fm.dtype, device=fm.device, memory_format=cl)
    _dev_call("pv_decoder_tail_f16", None, fm, fm.data_ptr(), img.data_ptr(), w1.data_ptr(), b1.data_ptr(),
              w2.data_ptr(), b2.data_ptr(), out.data_ptr(), n, h, w, cout, float(slope))
    return out


def _conv(x, c: nn.Conv2d):
    """The convolution alone (MIOpen); its folded bias goes to the epilogue."""
    return F.conv2d(x, c.weight, None, c.stride, c.padding, c.dilation, c.groups)


class PVNetInference(nn.Module):
    """Channels-last inference form of a :class:`PVNet` (fp16: configs[2]'s
    backbone; f32: configs[1]'s): BatchNorm folded into the convolutions
    (:func:`fold_batchnorm`); after each MIOpen convolution one HIP epilogue
    pass does the bias, the residual add and the activation
    (:func:`conv_epilogue`; the ReLU / residual / bias passes of the module
    form are gone, and fc's epilogue writes the concatenation with x8s
    itself); each decoder upsampling fused with the concatenation after it
    (:func:`upsample2x_cat`); the last concatenation (32 + 3 channels)
    zero-padded to 40 channels with ``convraw``'s first convolution given 5
    zero input channels; convraw's LeakyReLU and 1x1 convolution one HIP pass
    (:func:`head`) -- the same function up to rounding (MR:64-79).  Input: a
    channels_last float16 / float32 CUDA batch."""

    def __init__(self, net: PVNet):
        super().__init__()
        f = fold_batchnorm(net)
        self.seg_dim = f.seg_dim
        self.resnet18_8s, self.conv8s, self.conv4s, self.conv2s = f.resnet18_8s, f.conv8s, f.conv4s, f.conv2s
        c0 = f.convraw[0]
        self.raw_pad = (c0.in_channels + 7) // 8 * 8          # 35 -> 40 for the reference's dims
        pad = nn.Conv2d(self.raw_pad, c0.out_channels, c0.kernel_size, c0.stride, c0.padding, bias=True,
                        device=c0.weight.device, dtype=c0.weight.dtype)
        with torch.no_grad():
            pad.weight.zero_()
            pad.weight[:, :c0.in_channels] = c0.weight
            pad.bias.copy_(c0.bias)
        self.convraw = nn.Sequential(pad, *list(f.convraw)[1:])
        self.raw_in = c0.in_channels
        # fp16: convraw's input built and consumed inside one matrix-core kernel (decoder_tail)
        # when its shapes are the reference's (35 -> 32 -> 20 / 44); False = the MIOpen form
        # fp16: layer3 / layer4 / fc's 3x3 convolutions + epilogues as pv_conv3x3_f16
        self.fused_conv = True
        # fp16: a BasicBlock's 1x1 downsample summed into its conv2 (pv_conv3x3_ex_f16), conv8s reading
        # [xfc, x8s] from the two maps; False = the downsample as its own convolution + a residual read
        self.fused_ds = True
        self.fused_tail = (c0.in_channels == 35 and c0.out_channels == 32 and f.convraw[3].out_channels in (20, 44)
                           and self.conv2s[0].out_channels == 32)
        self.eval()

    def _wide(self, c: nn.Conv2d, x, kind="wide"):
        """fp16 and a 3x3 convolution one of the matrix-core kernels takes
        (kind "wide": pv_conv3x3_f16 -- layer2 / layer3 / layer4 / fc /
        conv8s; "c64": pv_conv64_f16 -- layer1): its weight in that kernel's
        layout, made once; else None (MIOpen + pv_conv_epilogue)."""
        ok = conv3x3_eligible(c) if kind == "wide" else conv64_eligible(c)
        if not (self.fused_conv and x.dtype == torch.float16 and ok):
            return None
        key = (c.weight.data_ptr(), c.weight.dtype, c.weight._version, kind)
        cache = self.__dict__.setdefault("_wide_w", {})
        hit = cache.get(id(c))
        if hit is None or hit[0] != key:
            hit = (key, conv3x3_weight(c) if kind == "wide" else conv64_weights(c))
            cache[id(c)] = hit
        return hit[1]

    def _conv_act(self, c: nn.Conv2d, x, act, res=None, rbias=None):
        if rbias is None and act in ("none", "relu"):
            w = self._wide(c, x, "c64")
            if w is not None:
                return conv64(x, w, c.bias, act, res=res)
        w = self._wide(c, x)
        if w is not None:
            if c.stride[0] != 1:
                if res is not None:
                    return conv_epilogue(_conv(x, c), c.bias, act, res=res, rbias=rbias)
                return conv3x3_ex(x, w, c.bias, c.dilation[0], stride=c.stride[0], act=act)
            return conv3x3(x, w, c.bias, c.dilation[0], act, res=res, rbias=rbias)
        return conv_epilogue(_conv(x, c), c.bias, act, res=res, rbias=rbias)

    def _conv_ds(self, c: nn.Conv2d, ds: nn.Conv2d, y, x):
        """conv2 of a BasicBlock with a downsample: ReLU(conv2(y) + b2 +
        ds(x) + bd) in one pv_conv3x3_ex_f16 pass (the 1x1 convolution
        summed into conv2's accumulator; RN:41-70), or None."""
        if not (self.fused_conv and y.dtype == torch.float16 and conv3x3_eligible(c) and c.stride == (1, 1)):
            return None
        key = (c.weight.data_ptr(), c.weight._version, ds.weight.data_ptr(), ds.weight._version, "ds")
        cache = self.__dict__.setdefault("_wide_w", {})
        hit = cache.get(id(c))
        if hit is None or hit[0] != key:
            hit = (key, conv3x3_weight(c, ds))
            cache[id(c)] = hit
        return conv3x3_ex(y, hit[1], c.bias, c.dilation[0], act="relu", x2=x, mode2="1x1", s2=ds.stride[0],
                          rbias=ds.bias)

    def _block(self, blk: BasicBlock, x):
        y = self._conv_act(blk.conv1, x, "relu")
        if blk.downsample is None:
            res, rb = x, None
        else:
            if self.fused_ds and downsample_eligible(blk.downsample):
                out = self._conv_ds(blk.conv2, blk.downsample[0], y, x)
                if out is not None:
                    return out
            res, rb = _conv(x, blk.downsample[0]), blk.downsample[0].bias
        return self._conv_act(blk.conv2, y, "relu", res=res, rbias=rb)

    def forward_modules(self, x):
        """The previous inference form (module epilogues: ATen bias / residual /
        activation passes after each convolution) -- A/B reference only."""
        x2s, x4s, x8s, _, _, xfc = self.resnet18_8s(x)
        fm = self.conv8s(torch.cat([xfc, x8s], 1))
        fm = self.conv4s(upsample2x_cat(fm, x4s, fm.shape[1] + x4s.shape[1]))
        fm = self.conv2s(upsample2x_cat(fm, x2s, fm.shape[1] + x2s.shape[1]))
        x = self.convraw(upsample2x_cat(fm, x, self.raw_pad))
        return x[:, :self.seg_dim], x[:, self.seg_dim:]

    def forward(self, x):
        r = self.resnet18_8s
        mp = r.maxpool
        pool3 = (mp.kernel_size, mp.stride, mp.padding, mp.dilation, mp.ceil_mode) == (3, 2, 1, 1, False)
        if (self.fused_conv and x.dtype == torch.float16 and stem_eligible(r.conv1) and x.shape[2] % 2 == 0
                and x.shape[3] % 2 == 0):
            key = (r.conv1.weight.data_ptr(), r.conv1.weight._version, r.conv1.bias.data_ptr(), r.conv1.bias._version)
            if getattr(self, "_stem_key", None) != key:     # the kernel's weight layout, made once
                self._stem_w = stem_weights(r.conv1)
                self._stem_key = key
            if pool3:                                  # conv1 + bn + relu + maxpool in one pass
                x2s, y = stem_conv(x, self._stem_w, pool=True)
            else:
                x2s = stem_conv(x, self._stem_w)
                y = mp(x2s)
        elif pool3:
            x2s, y = relu_maxpool(_conv(x, r.conv1), r.conv1.bias)
        else:
            x2s = conv_epilogue(_conv(x, r.conv1), r.conv1.bias, "relu")
            y = mp(x2s)
        for blk in r.layer1:
            y = self._block(blk, y)
        x4s = y
        for blk in r.layer2:
            y = self._block(blk, y)
        x8s = y
        for layer in (r.layer3, r.layer4):
            for blk in layer:
                y = self._block(blk, y)
        # fc (conv + BN + ReLU, MR:22-26) and torch.cat([xfc, x8s], 1) (MR:66) in one epilogue
        wfc = self._wide(r.fc[0], y)
        c8 = self.conv8s[0]
        w8 = self._wide(c8, y) if wfc is not None and c8.stride == (1, 1) and self.fused_ds else None
        if w8 is not None and c8.in_channels == r.fc[0].out_channels + x8s.shape[1]:
            # conv8s over torch.cat([xfc, x8s], 1) (MR:66) read from the two maps: no concatenated copy
            c = r.fc[0]
            xfc = conv3x3(y, wfc, c.bias, c.dilation[0], "relu")
            fm = conv3x3_ex(xfc, w8, c8.bias, c8.dilation[0], act="leaky", x2=x8s, mode2="cat",
                            slope=self.conv8s[2].negative_slope)
        else:
            if wfc is not None:
                c = r.fc[0]
                cat8 = conv3x3(y, wfc, c.bias, c.dilation[0], "relu", extra=x8s.shape[1])
                cat8[:, c.out_channels:].copy_(x8s)
            else:
                cat8 = conv_epilogue(_conv(y, r.fc[0]), r.fc[0].bias, "relu", skip=x8s)
            fm = self._conv_act(self.conv8s[0], cat8, "leaky")
        c4 = self.conv4s[0]
        if (fm.dtype == torch.float16 and self.fused_conv and fm.shape[1] == 128 and x4s.shape[1] == 64
                and c4.in_channels == 192 and c4.out_channels == 64 and c4.kernel_size == (3, 3)):
            key = (c4.weight.data_ptr(), c4.weight._version, c4.bias.data_ptr(), c4.bias._version)
            if getattr(self, "_c4s_key", None) != key:
                self._c4s_w = decoder_conv4s_weights(c4)
                self._c4s_key = key
            fm = decoder_conv4s(fm, x4s, self._c4s_w, self.conv4s[2].negative_slope)
        else:
            fm = upsample2x_cat(fm, x4s, fm.shape[1] + x4s.shape[1])
            fm = conv_epilogue(_conv(fm, c4), c4.bias, "leaky")
        c2 = self.conv2s[0]
        if (fm.dtype == torch.float16 and self.fused_conv and fm.shape[1] == 64 and x2s.shape[1] == 64
                and c2.in_channels == 128 and c2.out_channels == 32 and c2.kernel_size == (3, 3)):
            key = (c2.weight.data_ptr(), c2.weight._version, c2.bias.data_ptr(), c2.bias._version)
            if getattr(self, "_c2s_key", None) != key:     # the kernel's weight layout, made once
                self._c2s_w = decoder_conv2s_weights(c2)
                self._c2s_key = key
            fm = decoder_conv2s(fm, x2s, self._c2s_w, self.conv2s[2].negative_slope)
        else:
            fm = upsample2x_cat(fm, x2s, fm.shape[1] + x2s.shape[1])
            fm = conv_epilogue(_conv(fm, c2), c2.bias, "leaky")
        c0, c1 = self.convraw[0], self.convraw[3]
        slope = self.convraw[2].negative_slope
        if x.dtype == torch.float16 and self.fused_tail:
            key = (c0.weight.data_ptr(), c0.weight._version, c0.bias.data_ptr(), c0.bias._version,
                   c1.weight.data_ptr(), c1.weight._version, c1.bias.data_ptr(), c1.bias._version)
            if getattr(self, "_tail_key", None) != key:     # matrix-core layouts of convraw's weights, made once
                self._tail_w = decoder_tail_weights(c0, c1, self.raw_in)
                self._tail_key = key
            if self.seg_dim == 2 and TAIL_SPLIT:   # seg and ver as two dense maps (pv_decoder_tail_split_f16)
                return decoder_tail(fm, x, self._tail_w, slope, split=True)
            out = decoder_tail(fm, x, self._tail_w, slope)
            return out[:, :self.seg_dim], out[:, self.seg_dim:]
        fm = upsample2x_cat(fm, x, self.raw_pad)
        if not (c0.out_channels == 32 and c1.out_channels in (20, 44)):
            # pv_head_f16/_f32 take 32 -> 20 / 44 (the reference's two heads); other
            # PVNet(ver_dim, seg_dim, raw_dim) shapes run convraw's modules
            out = self.convraw(fm)
            return out[:, :self.seg_dim], out[:, self.seg_dim:]
        key = (c0.bias.data_ptr(), c0.bias._version, c1.weight.data_ptr(), c1.weight._version, c1.bias.data_ptr(),
               c1.bias._version, c1.weight.dtype)
        if getattr(self, "_head_key", None) != key:     # f32 copies of the head's parameters, made once
            self._head_w = (c0.bias.detach().float().contiguous(),
                            c1.weight.detach().float().reshape(c1.out_channels, -1).contiguous(),
                            c1.bias.detach().float().contiguous())
            self._head_key = key
        out = head(_conv(fm, c0), *self._head_w, slope=slope)
        return out[:, :self.seg_dim], out[:, self.seg_dim:]
