"""Debug: the vote kernel's per-wave phase cycles (PVV_TRACE build: run with
PVVOTE_LIB=variants/trace.so, built by `python tools/build_variant.py trace
-DPVV_TRACE`) on the synthetic headline field and on frames of the
random-init network's fp16 outputs (the configs[2] e2e inputs), one image
per call: segment setup, staging, hot loop, band re-check, exact flush,
exact-only hypotheses, and the flagged-MFMA count.  GPU only; not part of
the product or the tests."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, synth  # noqa: E402
from pvnet_amd.network import PVNet, PVNetInference  # noqa: E402
from pvnet_amd.ransac_voting_gpu import ransac_voting_layer_v3_from_network as v3  # noqa: E402

L = _lib.load()
L.pv_debug_set_vote_trace.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
buf = torch.zeros(16384 * 8, dtype=torch.int64, device=dev)


def traced(seg, ver, warm=50):
    L.pv_debug_set_vote_trace(None)
    for _ in range(warm):
        v3(seg, ver, 512)
    buf.zero_()
    L.pv_debug_set_vote_trace(ctypes.c_void_p(buf.data_ptr()))
    v3(seg, ver, 512)
    torch.cuda.synchronize()
    L.pv_debug_set_vote_trace(None)
    t = buf[:65536].view(-1, 8).cpu().numpy()
    live = t[:, 0] > 0
    c = buf[65536:].view(-1, 8).cpu().numpy()[: len(t)][live]
    t = t[live]
    span = (t[:, 1].max() - t[:, 0].min()) / 100.0
    nfix = t[:, 3] & 0xffffffff
    names = ["seg", "stage", "hot", "fix", "band", "flush", "xo"]
    tot = c[:, :7].sum(0)
    d = dict(zip(names, (tot / len(t)).round(0).tolist()))
    d["queued_pairs"] = round(float(c[:, 7].mean()), 2)
    return span, d, float(nfix.mean())


f = synth.synthetic_field(1234)
s, d, nf = traced(torch.from_numpy(f["seg"]).to(dev), torch.from_numpy(f["vertex"]).to(dev))
print(f"synthetic S(1234): span {s:.2f} us, cycles per wave {d}, flagged MFMAs per wave {nf:.1f}")
torch.manual_seed(0)
net = PVNetInference(PVNet(18, 2).eval()).to(dev).half().to(memory_format=torch.channels_last)
x = torch.randn(4, 3, 480, 640, device=dev).half().contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    seg, ver = net(x)
for i in range(2):
    s, d, nf = traced(seg[i:i + 1], ver[i:i + 1])
    print(f"network frame {i}: span {s:.2f} us, cycles per wave {d}, flagged MFMAs per wave {nf:.1f}")
