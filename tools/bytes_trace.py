"""Debug: phase stamps (s_memrealtime, 100 MHz) of the byte-output vote
kernel's first item per wave: 0 entry, 1 pixels loaded, 2 reductions, 3
records, 4 wave end.  GPU only."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, synth  # noqa: E402
from pvnet_amd import ransac_voting as rv  # noqa: E402

L = _lib.load()
L.pv_debug_set_bytes_trace.argtypes = [ctypes.c_void_p]
f = synth.synthetic_field(1234)
m = np.argmax(f["seg"][0], 0) == 1
rows, cols = np.nonzero(m)
VN, hn = 9, 512
coords = torch.from_numpy(np.stack([cols, rows], 1).astype(np.float32)).cuda()
direct = torch.from_numpy(np.ascontiguousarray(
    f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows, cols].transpose(2, 0, 1))).cuda()
tn = coords.shape[0]
idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
hyp = rv.generate_hypothesis(direct, coords, idxs)
inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
buf = torch.zeros(8 * 16384, dtype=torch.int64, device="cuda")
for it in range(3):
    buf.zero_()
    L.pv_debug_set_bytes_trace(ctypes.c_void_p(buf.data_ptr()) if it == 2 else None)
    rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
    torch.cuda.synchronize()
t = buf.view(-1, 8).cpu().numpy()[:, :5]
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
us = (t - t0) / 100.0
print("waves", len(t))
names = ["entry", "loaded", "reduced", "records", "end"]
for k in range(5):
    q = np.percentile(us[:, k], [0, 10, 50, 90, 100])
    print(f"{names[k]:8s}", " ".join(f"{v:7.2f}" for v in q))
for k in range(1, 5):
    d = us[:, k] - us[:, k - 1]
    q = np.percentile(d, [0, 10, 50, 90, 100])
    print(f"d{names[k]:7s}", " ".join(f"{v:7.2f}" for v in q))
