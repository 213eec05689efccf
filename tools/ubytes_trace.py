"""Per-wave phase stamps of k_vote_bytes_mfma (pv_debug_set_bytes_utrace) on the
U1 call (S(1234), hn=512, tn=29,861): wave start, end of the block's staging,
end; staging / work durations, block rounds per CU.  GPU only."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd import ransac_voting as rv  # noqa: E402
from pvnet_amd import synth  # noqa: E402

L = _lib.load()
L.pv_debug_set_bytes_utrace.argtypes = [ctypes.c_void_p]
VN, hn = 9, 512
f = synth.synthetic_field(1234)
m = np.argmax(f["seg"][0], 0) == 1
rows, cols = np.nonzero(m)
tn = len(rows)
coords = torch.from_numpy(np.stack([cols, rows], 1).astype(np.float32)).cuda()
direct = torch.from_numpy(np.ascontiguousarray(
    f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows, cols].transpose(2, 0, 1))).cuda()
idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
hyp = rv.generate_hypothesis(direct, coords, idxs)
inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
buf = torch.zeros(16384 * 4 * 4, dtype=torch.int64, device="cuda")
for it in range(4):
    buf.zero_()
    L.pv_debug_set_bytes_utrace(ctypes.c_void_p(buf.data_ptr() if it == 3 else 0))
    rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
    torch.cuda.synchronize()
L.pv_debug_set_bytes_utrace(ctypes.c_void_p(0))
t = buf.view(-1, 4).cpu().numpy()
t = t[t[:, 0] > 0]
s, st, e, hw = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
t0 = s.min()
print("waves", len(t), "span us", (e.max() - t0) / 100.0)
for name, x in (("start", (s - t0) / 100), ("staging", (st - s) / 100), ("work", (e - st) / 100),
                ("end", (e - t0) / 100), ("life", (e - s) / 100)):
    q = np.percentile(x, [0, 1, 10, 50, 90, 99, 100])
    print(f"{name:8s}", " ".join(f"{v:7.2f}" for v in q))
hist, edges = np.histogram((s - t0) / 100, bins=24)
print("start histogram:", list(zip(np.round(edges[:-1], 1).tolist(), hist.tolist())))
hist, edges = np.histogram((e - t0) / 100, bins=24)
print("end histogram:", list(zip(np.round(edges[:-1], 1).tolist(), hist.tolist())))
xcc = (hw >> 32) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
cuid = xcc * 64 + se * 16 + cu
ids, cnt = np.unique(cuid, return_counts=True)
print("waves per CU:", dict(zip(*np.unique(cnt, return_counts=True))))
ce = np.array([e[cuid == c].max() for c in ids])
print("CU last end percentiles:", np.round(np.percentile((ce - t0) / 100, [0, 25, 50, 75, 100]), 2).tolist())
busy = np.array([((e - s)[cuid == c]).sum() for c in ids]) / 100 / 12
print("CU summed wave life / 12 slots, us percentiles:", np.round(np.percentile(busy, [0, 50, 100]), 2).tolist())
