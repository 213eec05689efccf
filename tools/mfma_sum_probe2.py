"""Characterise the matrix core's f32 sum of 8 fp16 products
(v_mfma_f32_32x32x8_f16, zero accumulator; pv_debug_mfma_sums) where
tests/test_gpu_vote_mfma.py found errors far above 16 u sum|terms|: tiny
products and fp16 subnormal operands.  For each family, the worst error
relative to u*sum|terms| and to max|term|, and the worst absolute error."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_vote_mfma import crafted_tiles, mfma_sums, U

dev = torch.device("cuda:0")


def stats(A, B, name):
    D = mfma_sums(A, B, dev).astype(np.float64)
    t = A.astype(np.float64)[:, :, :, None] * B.astype(np.float64)[:, None, :, :]
    exact = t.astype(np.longdouble).sum(axis=2)
    mag = np.abs(t).sum(axis=2)
    mx = np.abs(t).max(axis=2)
    err = np.abs(D.astype(np.longdouble) - exact).astype(np.float64)
    ok = mag > 0
    r1 = (err[ok] / mag[ok] / U).max()
    r2 = (err[ok] / mx[ok]).max()
    i = np.argmax(np.where(ok, err / np.where(ok, mag, 1), 0))
    print(f"{name:40s} max err/(u sum|t|) {r1:9.2f}  max err/max|t| 2^{np.log2(r2 + 1e-300):6.1f}  "
          f"max abs err 2^{np.log2(err.max() + 1e-300):6.1f}  (sum|t| there 2^{np.log2(mag.ravel()[i] + 1e-300):6.1f})")


rng = np.random.default_rng(7)
A0, B0 = crafted_tiles(rng, 256)
sel = np.arange(256) % 4 == 0          # family 0: one big + 7 near-ulp smalls, normal operands
A0, B0 = A0[sel], B0[sel]
for k in (0, 4, 8, 12, 14, 16, 18, 20, 24):
    A = (A0.astype(np.float64) * 2.0 ** -k).astype(np.float16)     # smalls become subnormal from k ~ 2
    stats(A, B0, f"family0 A*2^-{k}")
for k in (0, 4, 8, 12, 16):
    B = (B0.astype(np.float64) * 2.0 ** -k).astype(np.float16)
    stats(A0, B, f"family0 B*2^-{k}")
# all-normal operands, tiny products: A, B in [2^-14, 2^-13)
A = (rng.uniform(1, 2, (64, 32, 8)) * rng.choice([-1, 1], (64, 32, 8)) * 2.0 ** -14).astype(np.float16)
B = (rng.uniform(1, 2, (64, 8, 32)) * rng.choice([-1, 1], (64, 8, 32)) * 2.0 ** -14).astype(np.float16)
stats(A, B, "normal operands, products ~2^-28")
for e in (-20, -10, 0, 10):
    A = (rng.uniform(1, 2, (64, 32, 8)) * rng.choice([-1, 1], (64, 32, 8)) * 2.0 ** (e // 2)).astype(np.float16)
    B = (rng.uniform(1, 2, (64, 8, 32)) * rng.choice([-1, 1], (64, 8, 32)) * 2.0 ** (e - e // 2)).astype(np.float16)
    stats(A, B, f"random signs, products ~2^{e}")
# one subnormal operand per product, products large
A = (rng.uniform(1, 1024, (64, 32, 8)) * rng.choice([-1, 1], (64, 32, 8)) * 2.0 ** -24).astype(np.float16)
B = (rng.uniform(1, 2, (64, 8, 32)) * 2.0 ** rng.integers(0, 15, (64, 8, 32))).astype(np.float16)
stats(A, B, "subnormal A x large B")
# mixed: half the products tiny (subnormal x normal), half ~1
A = (rng.uniform(1, 2, (64, 32, 8)) * rng.choice([-1, 1], (64, 32, 8))).astype(np.float16)
A[:, :, ::2] = (rng.uniform(1, 1024, (64, 32, 4)) * 2.0 ** -24).astype(np.float16)
B = (rng.uniform(1, 2, (64, 8, 32)) * rng.choice([-1, 1], (64, 8, 32))).astype(np.float16)
stats(A, B, "alternating subnormal/normal A")
