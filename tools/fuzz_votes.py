"""Randomised parity sweep of the API vote kernels against the C oracle:
voting_for_hypothesis (dense with both byte kernels, and OR) and vote_counts
(k_vote_mfma when hn is a multiple of 512's groups, else k_vote_count) over
random tn / vn / hn / thresholds / coordinate spans / degenerate pixels and
hypotheses.  GPU only; prints one line per case and a summary, exits 1 on the
first mismatch (the case's parameters are printed)."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd import ransac_voting as rv  # noqa: E402

L = _lib.load()
L.pv_debug_set_bytes_mfma.argtypes = [ctypes.c_int32]
L.pv_debug_set_bytes_mfma.restype = ctypes.c_int32
budget = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
dev = torch.device("cuda:0")
t_end = time.time() + budget
case = 0
while time.time() < t_end:
    rng = np.random.default_rng(case)
    tn = int(rng.integers(1, 4000))
    vn = int(rng.integers(1, 5))
    hn = int(rng.choice([1, 7, 64, 100, 128, 200, 512, 513]))
    span = float(rng.choice([8.0, 640.0, 5000.0, 50000.0]))
    thr = float(rng.choice([0.99, 0.9, 0.5, 0.3, 0.999, 0.9999]))
    coords = (rng.random((tn, 2)) * span).astype(np.float32)
    if rng.random() < 0.5:
        coords = np.round(coords)
    ang = rng.uniform(-np.pi, np.pi, (tn, vn))
    scale = rng.choice([1.0, 1e-7, 0.0, 1e5, 2e19], size=(tn, vn), p=[0.96, 0.01, 0.01, 0.01, 0.01])
    direct = np.stack([np.cos(ang) * scale, np.sin(ang) * scale], -1).astype(np.float32)
    hyp = (rng.random((hn, vn, 2)) * span * 1.4 - span * 0.2).astype(np.float32)
    k = rng.random((hn, vn))
    hyp[k < 0.02] = coords[rng.integers(0, tn, (int((k < 0.02).sum()),))]
    hyp[(k >= 0.02) & (k < 0.03)] = 3e7
    if thr in (0.99, 0.9) and rng.random() < 0.5:   # a threshold exactly on a reference cosine
        i, h = int(rng.integers(0, tn)), int(rng.integers(0, hn))
        d = hyp[h, 0] - coords[i]
        n = direct[i, 0]
        c = float(np.float32(np.dot(d, n) / (np.linalg.norm(d) * np.linalg.norm(n) + 1e-30)))
        if 0.05 < c < 0.999999:
            thr = c
    ref = np.zeros((hn, vn, tn), np.uint8)
    O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
    dd, cc, hh = (torch.from_numpy(a).to(dev) for a in (direct, coords, hyp))
    for name, mfma, dense in (("valu-dense", 0, True), ("mfma-dense", 1, True), ("or", 0, False)):
        prev = L.pv_debug_set_bytes_mfma(mfma)
        init = np.zeros_like(ref) if dense else (rng.random(ref.shape) < 0.1).astype(np.uint8) * 5
        out = torch.from_numpy(init.copy()).to(dev)
        (rv.voting_for_hypothesis_dense if dense else rv.voting_for_hypothesis)(dd, cc, hh, out, thr)
        L.pv_debug_set_bytes_mfma(prev)
        exp = ref if dense else np.where(ref == 1, 1, init).astype(np.uint8)
        got = out.cpu().numpy()
        if not np.array_equal(got, exp):
            bad = np.argwhere(got != exp)
            print(f"MISMATCH {name} case={case} tn={tn} vn={vn} hn={hn} span={span} thr={thr!r}: "
                  f"{len(bad)} bytes, first {bad[:3].tolist()}", flush=True)
            sys.exit(1)
    cnt = rv.vote_counts(dd, cc, hh, thr).cpu().numpy()
    if not np.array_equal(cnt, ref.sum(2)):
        print(f"MISMATCH counts case={case} tn={tn} vn={vn} hn={hn} span={span} thr={thr!r}", flush=True)
        sys.exit(1)
    case += 1
    if case % 20 == 0:
        print(f"{case} cases ok", flush=True)
print(f"fuzz: {case} cases, every byte and count equal to the oracle's")
