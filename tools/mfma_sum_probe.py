"""Worst cases of the matrix core's 8-product sums (pv_debug_mfma_sums):
prints the terms, the exact sum and the device result of the largest errors
relative to u * sum|terms| for each crafted family of
tests/test_gpu_vote_mfma.py."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_vote_mfma import crafted_tiles, mfma_sums, U

dev = torch.device("cuda:0")
rng = np.random.default_rng(2024)
A, B = crafted_tiles(rng, 512)
D = mfma_sums(A, B, dev).astype(np.float64)
t = A.astype(np.float64)[:, :, :, None] * B.astype(np.float64)[:, None, :, :]
exact = t.astype(np.longdouble).sum(axis=2)
mag = np.abs(t).sum(axis=2)
err = np.abs(D.astype(np.longdouble) - exact).astype(np.float64)
ratio = np.where(mag > 0, err / np.where(mag > 0, mag, 1) / U, 0)
for fam in range(4):
    r = ratio[fam::4]
    idx = np.argsort(r.ravel())[::-1][:5]
    for k in idx:
        ti, row, col = np.unravel_index(k, r.shape)
        i = fam + 4 * ti
        terms = t[i, row, :, col]
        print(f"fam {fam} tile {i} r{row} c{col}: ratio {r[ti, row, col]:.2f}  dev {D[i, row, col]!r}  exact {float(exact[i, row, col])!r}")
        print("   A", [float(x) for x in A[i, row]], "\n   B", [float(x) for x in B[i, :, col]])
        print("   terms", [float(x) for x in terms])
