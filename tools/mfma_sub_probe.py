"""How v_mfma_f32_32x32x8_f16 multiplies fp16 subnormal operands
(pv_debug_mfma_sums): single products and a subnormal product beside a
normal one, relative error per product."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_vote_mfma import mfma_sums

dev = torch.device("cuda:0")
rng = np.random.default_rng(3)
T = 64
# 1. one nonzero product per sum: A subnormal (m * 2^-24, m in 1..1023), B normal random
A = np.zeros((T, 32, 8), np.float16)
B = np.zeros((T, 8, 32), np.float16)
k = rng.integers(0, 8, T)
for i in range(T):
    A[i, :, k[i]] = (rng.integers(1, 1024, 32) * 2.0 ** -24).astype(np.float16)
    B[i, k[i], :] = (rng.uniform(1, 2, 32) * 2.0 ** rng.integers(-14, 15, 32) * rng.choice([-1, 1], 32)).astype(np.float16)
D = mfma_sums(A, B, dev)
t = (A.astype(np.float64)[:, :, :, None] * B.astype(np.float64)[:, None, :, :]).sum(2)
rel = np.abs(D - t) / np.abs(t)
print(f"1 product, subnormal x normal: exact {np.mean(D == t):.4f}, max rel err 2^{np.log2(rel.max() + 1e-300):.1f}")
# by the subnormal's leading bit
m = (A.astype(np.float64).max(2) / 2.0 ** -24).astype(int)      # [T, 32]
for lb in range(10):
    sel = (m >= 2 ** lb) & (m < 2 ** (lb + 1))
    r = rel[np.broadcast_to(sel[:, :, None], rel.shape)]
    print(f"   subnormal m in [2^{lb}, 2^{lb + 1}): max rel err 2^{np.log2(r.max() + 1e-300):.1f}  exact {np.mean(r == 0):.3f}")
# 2. both subnormal? (subnormal x subnormal underflows f32? no: >= 2^-48)
A2 = (rng.integers(1, 1024, (T, 32, 8)) * 2.0 ** -24).astype(np.float16)
B2 = (rng.integers(1, 1024, (T, 8, 32)) * 2.0 ** -24).astype(np.float16)
A2[:, :, 1:] = 0
D2 = mfma_sums(A2, B2, dev)
t2 = (A2.astype(np.float64)[:, :, :, None] * B2.astype(np.float64)[:, None, :, :]).sum(2)
print(f"1 product, subnormal x subnormal: exact {np.mean(D2 == t2):.4f}, max rel {np.log2((np.abs(D2 - t2) / t2).max() + 1e-300):.1f}")
# 3. a normal product ~1 beside one subnormal product of size 2^-j
for j in (4, 8, 12, 16, 20):
    A3 = np.zeros((T, 32, 8), np.float16)
    B3 = np.zeros((T, 8, 32), np.float16)
    A3[:, :, 0] = (rng.uniform(1, 2, (T, 32))).astype(np.float16)
    B3[:, 0, :] = (rng.uniform(0.5, 1, (T, 32))).astype(np.float16)
    A3[:, :, 1] = (rng.integers(1, 1024, (T, 32)) * 2.0 ** -24).astype(np.float16)
    B3[:, 1, :] = (rng.uniform(1, 2, (T, 32)) * 2.0 ** (14 - j)).astype(np.float16)
    D3 = mfma_sums(A3, B3, dev)
    tt = A3.astype(np.float64)[:, :, :, None] * B3.astype(np.float64)[:, None, :, :]
    ex = tt.sum(2)
    small = np.abs(tt[:, :, 1, :])
    e = np.abs(D3 - ex)
    print(f"normal ~1 + subnormal product ~2^-{j}: max err 2^{np.log2(e.max() + 1e-300):.1f}, max err/small "
          f"2^{np.log2((e / small).max() + 1e-300):.1f}, max err/(u*sum) {(e / np.abs(tt).sum(2) / 2.0 ** -24).max():.2f}")
