"""Debug: phase stamps of the compaction blocks (0 start, 1 totals, 2 mask
scan, 3 end), relative to the earliest start, in microseconds.  GPU only."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, synth  # noqa: E402
from pvnet_amd.ransac_voting_gpu import ransac_voting_layer_v3_from_network  # noqa: E402

L = _lib.load()
L.pv_debug_compact_trace.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
f = synth.synthetic_field(1234)
seg = torch.from_numpy(f["seg"]).cuda()
vert = torch.from_numpy(f["vertex"]).cuda()
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 400):
    ransac_voting_layer_v3_from_network(seg, vert, 512)
torch.cuda.synchronize()
L.pv_debug_compact_trace(1, None, 0)
ransac_voting_layer_v3_from_network(seg, vert, 512)
torch.cuda.synchronize()
L.pv_debug_compact_trace(0, None, 0)
buf = np.zeros(4096 * 4, np.uint64)
L.pv_debug_compact_trace(0, buf.ctypes.data, buf.size)
t = buf.reshape(-1, 4).astype(np.int64)
t = t[t[:, 0] > 0]
us = (t - t[:, 0].min()) / 100.0
print("blocks", len(t))
for k, name in enumerate(["start", "totals", "scan", "end"]):
    q = np.percentile(us[:, k], [0, 10, 50, 90, 100])
    print(f"{name:7s}", " ".join(f"{v:7.2f}" for v in q))
