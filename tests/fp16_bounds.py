"""Elementwise error bounds for the fp16 convolution kernels against an fp32
convolution of the same fp16 inputs (tests/test_backbone.py).

A kernel's output differs from the fp32 reference only by
  * the f32 accumulation order: the products of fp16 operands are exact in
    f32, and any order of K - 1 f32 additions (the matrix core's included,
    DESIGN.md 5a measures its sums within 16 u per 8 products) stays within
    2 K u32 sum|terms| here -- sum|terms| = conv(|x|, |w|);
  * each fp16 rounding of the epilogue (the convolution's output, the bias
    add, the residual add, the LeakyReLU product): half an fp16 ulp of the
    rounded value, taken at |reference value| + the error carried so far, so
    the bound holds for the kernel's own intermediate;
  * in the decoder kernels, the x2 bilinear blend done in fp16 (weights
    rounded to fp16, two roundings per blend, two separable blends): at most
    3 * 2^-10 of the largest |fm| among the blended source pixels, propagated
    through the convolution by sum |w|.
ReLU is 1-Lipschitz and exact; LeakyReLU's slope is < 1.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

U32 = 2.0 ** -24
BLEND = 3 * 2.0 ** -10 * 1.01


def hulp(v: torch.Tensor) -> torch.Tensor:
    """Half an fp16 ulp at magnitude |v| (f64): the largest error of rounding a
    real of that magnitude to fp16 (2^-25 below the normal range)."""
    a = v.abs().double().clamp_min(2.0 ** -14)
    return torch.exp2(torch.floor(torch.log2(a)) - 11)


def conv64(x: torch.Tensor, w: torch.Tensor, **conv) -> torch.Tensor:
    """The reference: F.conv2d in f64 (ATen's own im2col + GEMM path; MIOpen's
    algorithms, e.g. Winograd, are not used) of the fp16 inputs."""
    with torch.backends.cudnn.flags(enabled=False):
        return F.conv2d(x.double(), w.double(), None, **conv)


def acc_bound(x: torch.Tensor, w: torch.Tensor, k: int, **conv) -> torch.Tensor:
    """2 k u32 * conv(|x|, |w|) in f64 (k = products per output)."""
    return 2 * k * U32 * conv64(x.abs(), w.abs(), **conv)


def round_step(v: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """Error after rounding a value near v (within e of it) to fp16."""
    return e + hulp(v.double().abs() + e)


def leaky_step(v: torch.Tensor, e: torch.Tensor, slope: float) -> torch.Tensor:
    """Error after LeakyReLU(slope) with the negative side's product rounded to fp16."""
    return e + torch.where(v < e, hulp(slope * (v.double().abs() + e)), torch.zeros_like(e))


def blend_source_max(fm: torch.Tensor) -> torch.Tensor:
    """For the x2 align_corners upsampling of fm [n, c, h, w]: an upper bound
    of |fm| over the source pixels each output pixel blends (the 3 x 3
    neighbourhood of its nearest source pixel covers them), [n, c, 2h, 2w] f64."""
    m = F.max_pool2d(fm.double().abs(), 3, 1, 1)
    return F.interpolate(m, scale_factor=2, mode="nearest")


def check(got: torch.Tensor, ref: torch.Tensor, bound: torch.Tensor, name: str) -> float:
    """Assert |got - ref| <= bound elementwise; returns the largest ratio."""
    d = (got.double() - ref.double()).abs()
    r = float((d / bound.clamp_min(1e-300)).max())
    print(f"{name}: vs fp32 conv of the same fp16 inputs: max |dev| {float(d.max()):.3e}, "
          f"largest dev / bound {r:.3f} (bound median {float(bound.median()):.2e})")
    assert bool((d <= bound).all()), f"{name}: {int((d > bound).sum())} elements outside the fp32 bound"
    return r
