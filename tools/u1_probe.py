"""Debug: voting_for_hypothesis (dense bytes) time vs row alignment, and the
chip's plain write bandwidth for the same byte count.  GPU only."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import ransac_voting as rv  # noqa: E402
from pvnet_amd import synth  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


f = synth.synthetic_field(1234)
m = np.argmax(f["seg"][0], 0) == 1
rows, cols = np.nonzero(m)
VN = 9
import os
hn = int(os.environ.get('U1_HN', '512'))
for tn in (29861, 29824, 29696, 29860):
    coords = torch.from_numpy(np.stack([cols[:tn], rows[:tn]], 1).astype(np.float32)).cuda()
    direct = torch.from_numpy(np.ascontiguousarray(
        f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows[:tn], cols[:tn]].transpose(2, 0, 1))).cuda()
    idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
    hyp = rv.generate_hypothesis(direct, coords, idxs)
    inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
    ms = timeit(lambda: rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99))
    mz = timeit(lambda: inl.fill_(1))
    print(f"tn={tn} (mod 128 = {tn % 128}): vote {ms * 1e3:.1f} us = {inl.numel() / ms / 1e6:.0f} GB/s;"
          f" fill_ {mz * 1e3:.1f} us = {inl.numel() / mz / 1e6:.0f} GB/s")
