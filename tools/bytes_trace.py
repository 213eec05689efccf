"""Debug: per-wave phase stamps of k_vote_bytes (voting_for_hypothesis, dense)
from a library built with -DPVVOTE_TRACE_U1 (variants/u1trace.so):
start, end of the first segment, end; s_memrealtime at 100 MHz.  GPU only."""
import ctypes
import os
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
VN, tn, hn = 9, 29861, int(os.environ.get("U1_HN", "512"))
coords = torch.from_numpy(np.stack([cols, rows], 1).astype(np.float32)).cuda()
direct = torch.from_numpy(np.ascontiguousarray(
    f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows, cols].transpose(2, 0, 1))).cuda()
idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
hyp = rv.generate_hypothesis(direct, coords, idxs)
inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
buf = torch.zeros(65536 * 8, dtype=torch.int64, device="cuda")
for it in range(4):
    buf.zero_()
    L.pv_debug_set_bytes_trace(ctypes.c_void_p(buf.data_ptr() if it == 3 else 0))
    rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
    torch.cuda.synchronize()
t = buf.view(-1, 8).cpu().numpy()
t = t[t[:, 0] > 0]
s, f1, e, su, stg = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4]
t0 = s.min()
print("waves", len(t), "span us", (e.max() - t0) / 100.0)
for name, x in (("start", (s - t0) / 100), ("staged", (stg - s) / 100), ("setup", (su - s) / 100), ("first", (f1 - s) / 100),
                ("end", (e - t0) / 100), ("life", (e - s) / 100)):
    q = np.percentile(x, [0, 1, 10, 50, 90, 99, 100])
    print(f"{name:6s}", " ".join(f"{v:7.2f}" for v in q))
hist, edges = np.histogram((e - t0) / 100, bins=20)
print("end histogram:", list(zip(np.round(edges[:-1], 1).tolist(), hist.tolist())))
hist, edges = np.histogram((s - t0) / 100, bins=20)
print("start histogram:", list(zip(np.round(edges[:-1], 1).tolist(), hist.tolist())))
# the slowest waves' items (one item per wave: g fastest, then window, then keypoint)
nwin, nhg = (tn + 511) // 512, (hn + 63) // 64
idx = np.nonzero(buf.view(-1, 8).cpu().numpy()[:, 0] > 0)[0]
order = np.argsort(e)[::-1][:12]
for k in order:
    wv = idx[k]
    g, rest = wv % nhg, wv // nhg
    print(f"wave {wv}: v={rest % VN} w={(rest // VN + nwin - 1) % nwin} g={g}  setup {(su[k] - s[k]) / 100:.2f} loop_end {(f1[k] - s[k]) / 100:.2f} end {(e[k] - t0) / 100:.2f}")
# per-XCC / per-CU: does a CU's or an XCD's share of waves set its end time?
hw = t[:, 5]
xcc = (hw >> 32) & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
cuid = xcc * 64 + se * 16 + cu
end = (e - t0) / 100
print("end by XCC (n, median, p90, max):",
      [f"{k}: {(xcc == k).sum()} {np.median(end[xcc == k]):.2f} {np.percentile(end[xcc == k], 90):.2f} {end[xcc == k].max():.2f}"
       for k in range(8) if (xcc == k).any()])
ids, cnt = np.unique(cuid, return_counts=True)
print("waves per CU histogram:", dict(zip(*np.unique(cnt, return_counts=True))))
wpc = dict(zip(ids, cnt))
n_of = np.array([wpc[c] for c in cuid])
for n in sorted(set(n_of.tolist())):
    sel = n_of == n
    print(f"CUs with {n} waves: end median {np.median(end[sel]):.2f} p90 {np.percentile(end[sel], 90):.2f} max {end[sel].max():.2f}")
# per CU: last end vs first start
cu_end = {c: end[cuid == c].max() for c in ids}
v = np.array(list(cu_end.values()))
print("CU last-end percentiles:", np.round(np.percentile(v, [0, 10, 50, 90, 100]), 2).tolist())
# age: end by block-index quartile (blocks dispatch in index order)
bidx = idx // 4
qq = np.digitize(bidx, np.percentile(bidx, [25, 50, 75]))
print("end by block-index quartile (mean):", [f"{k}: {((e - t0) / 100)[qq == k].mean():.2f}" for k in range(4)])
