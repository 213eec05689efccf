"""Debug: phase stamps (s_memrealtime, 100 MHz) of k_refine_solve's blocks in
one traced v3 call after warm-up calls -- entry, argmax done, votes done,
partials reduced, partial published, (the image's gathering block) all
partials gathered and summed, solved; and when the block's pixels had
arrived -- relative to the first block's entry.  Needs a PVV_TRACE build:
    python tools/build_variant.py trace -DPVV_TRACE
    PVVOTE_LIB=variants/trace.so python tools/refine_trace.py
GPU only; not part of the product or the tests."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, synth  # noqa: E402
from pvnet_amd.ransac_voting_gpu import ransac_voting_layer_v3_from_network, VotingWorkspace  # noqa: E402

L = _lib.load()
L.pv_debug_set_refine_trace.argtypes = [ctypes.c_void_p]
f = synth.synthetic_field(1234)
seg = torch.from_numpy(f["seg"]).cuda()
vert = torch.from_numpy(f["vertex"]).cuda()
ws = VotingWorkspace()
buf = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
names = ["entry", "argmax", "votes", "reduced", "published", "gathered", "solved", "pixels"]
res = []
for trial in range(5):
    L.pv_debug_set_refine_trace(None)
    for it in range(200):
        ransac_voting_layer_v3_from_network(seg, vert, 512, _seed=it, _workspace=ws)
    buf.zero_()
    L.pv_debug_set_refine_trace(ctypes.c_void_p(buf.data_ptr()))
    ransac_voting_layer_v3_from_network(seg, vert, 512, _seed=7, _workspace=ws)
    torch.cuda.synchronize()
    L.pv_debug_set_refine_trace(None)
    t = buf.view(-1, 8).cpu().numpy().astype(np.float64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0
    us[t == 0] = np.nan
    res.append(us)
    print(f"trial {trial}: blocks {len(t)}", "  ".join(
        f"{nm} p50 {np.nanmedian(us[:, k]):.2f} max {np.nanmax(us[:, k]):.2f}" for k, nm in enumerate(names)
        if not np.all(np.isnan(us[:, k]))), flush=True)
