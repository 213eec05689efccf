"""Debug: per-wave start/end timestamps of the pipeline's vote kernel
(s_memrealtime, 100 MHz) -> when waves start, how long they live, how the
finish times spread.  GPU only; not part of the product or the tests."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, synth  # noqa: E402
from pvnet_amd.ransac_voting_gpu import ransac_voting_layer_v3_from_network  # noqa: E402

L = _lib.load()
L.pv_debug_set_vote_trace.argtypes = [ctypes.c_void_p]
f = synth.synthetic_field(1234)
seg = torch.from_numpy(f["seg"]).cuda()
vert = torch.from_numpy(f["vertex"]).cuda()
buf = torch.zeros(16384 * 8, dtype=torch.int64, device="cuda")
# warm clocks: many back-to-back calls without a sync, then the traced call
WARM = int(sys.argv[1]) if len(sys.argv) > 1 else 400
L.pv_debug_set_vote_trace(None)
for it in range(WARM):
    ransac_voting_layer_v3_from_network(seg, vert, 512)
buf.zero_()
L.pv_debug_set_vote_trace(ctypes.c_void_p(buf.data_ptr()))
ransac_voting_layer_v3_from_network(seg, vert, 512)
torch.cuda.synchronize()
L.pv_debug_set_vote_trace(None)
t = buf[:65536].view(-1, 8).cpu().numpy()
t = t[t[:, 0] > 0]
s, e, hw = t[:, 0], t[:, 1], t[:, 2]
nfix, nseg = t[:, 3] & 0xffffffff, t[:, 3] >> 32
t0 = s.min()
s_us, e_us = (s - t0) / 100.0, (e - t0) / 100.0
life = e_us - s_us
print("waves", len(t), "span us", e_us.max())
tl = (t[:, 4] - t0) / 100.0
print("first hot loop at (us): p10 %.2f p50 %.2f p90 %.2f max %.2f" % (*np.percentile(tl - s_us, [10, 50, 90]), (tl - s_us).max()))
for name, x in (("start", s_us), ("end", e_us), ("life", life)):
    q = np.percentile(x, [0, 1, 10, 50, 90, 99, 100])
    print(f"{name:6s}", " ".join(f"{v:7.2f}" for v in q))
# per-CU / SE breakdown of the start times (HW_ID: wave[3:0] simd[5:4] cu[11:8] se[14:13] on gfx9)
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
print("start by SE:", [f"{np.median(s_us[se == k]):.2f}" for k in range(8) if (se == k).any()])
xcc = (hw >> 32) & 0xF
print("life by XCC (median, p90, max):", [f"{k}: {np.median(life[xcc == k]):.2f} {np.percentile(life[xcc == k], 90):.2f} {life[xcc == k].max():.2f}" for k in range(8) if (xcc == k).any()])
cuid = xcc * 64 + se * 16 + cu
per_cu = {c: np.median(life[cuid == c]) for c in np.unique(cuid)}
v = np.array(list(per_cu.values()))
print("per-CU median life: min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f (%d CUs)" % (v.min(), *np.percentile(v, [10, 50, 90]), v.max(), len(v)))
simd = (hw >> 4) & 3
wid_in = cuid * 4 + simd
cnt = np.bincount(np.unique(wid_in, return_inverse=True)[1])
print("waves per SIMD: min", cnt.min(), "max", cnt.max())
hist, edges = np.histogram(s_us, bins=20)
print("start histogram:", hist.tolist(), "edges", np.round(edges[[0, -1]], 2).tolist())
hist, edges = np.histogram(e_us, bins=20)
print("end histogram:", hist.tolist(), "edges", np.round(edges[[0, -1]], 2).tolist())

life = e_us - s_us
for name, m in (("1 segment", nseg == 1), ("2 segments", nseg == 2), ("3+ segments", nseg >= 3)):
    if m.any():
        print(f"{name:12s} waves {m.sum():5d}  life median {np.median(life[m]):6.2f}  max {life[m].max():6.2f}")
print("fix steps per wave: median", np.median(nfix), "p90", np.percentile(nfix, 90), "max", nfix.max())
nslow, nxo = t[:, 5] >> 32, t[:, 5] & 0xffffffff
if (t[:, 6] > 0).all():
    tt = (t[:, 6] - t0) / 100.0 - s_us
    th = (t[:, 7] - t0) / 100.0 - s_us
    print("after the work split (us): p10 %.2f p50 %.2f p90 %.2f" % tuple(np.percentile(tt, [10, 50, 90])))
    print("after the hypotheses (us): p10 %.2f p50 %.2f p90 %.2f" % tuple(np.percentile(th, [10, 50, 90])))
print("slow sub-chunks per wave: mean", nslow.mean(), "max", nslow.max(), "| exact-only hypotheses per wave: mean", nxo.mean(), "max", nxo.max())
order = np.argsort(life)
for q in (0.1, 0.5, 0.9, 0.99):
    k = order[int(q * (len(order) - 1))]
    print(f"life q{q}: {life[k]:.2f} us nfix {nfix[k]} nseg {nseg[k]}")
top = order[-50:]
print("slowest 50: nfix mean", nfix[top].mean(), "nseg mean", nseg[top].mean(), " | all: nfix mean", nfix.mean(), "nseg mean", nseg.mean())
print("corr(life, nfix)", np.corrcoef(life, nfix)[0, 1], "corr(life, nseg)", np.corrcoef(life, nseg)[0, 1])
# per-SIMD: when its first and last wave end (equal work per wave: a wide
# gap means unfair issue within the SIMD, a wide spread of last ends means
# SIMDs of different speed)
first_end, last_end = [], []
for sid in np.unique(wid_in):
    e = e_us[wid_in == sid]
    first_end.append(e.min())
    last_end.append(e.max())
first_end, last_end = np.array(first_end), np.array(last_end)
print("per-SIMD last end: p10 %.2f p50 %.2f p90 %.2f max %.2f" % (*np.percentile(last_end, [10, 50, 90]), last_end.max()))
print("per-SIMD first end: p10 %.2f p50 %.2f p90 %.2f" % tuple(np.percentile(first_end, [10, 50, 90])))
gap = last_end - first_end
print("per-SIMD last-first gap: p10 %.2f p50 %.2f p90 %.2f max %.2f" % (*np.percentile(gap, [10, 50, 90]), gap.max()))
# Within each SIMD: is a wave's end set by its start order (age-ordered
# issue), by its hardware wave slot, or by its block's place in the grid?
uniq, inv = np.unique(wid_in, return_inverse=True)
srank = np.zeros(len(t), int)
for g in range(len(uniq)):
    idx = np.nonzero(inv == g)[0]
    srank[idx[np.argsort(s_us[idx], kind="stable")]] = np.arange(len(idx))
erel = e_us - np.array([e_us[inv == inv[i]].min() for i in range(len(t))])
print("end after the SIMD's first end, by start rank:",
      [f"{k}: {erel[srank == k].mean():.2f}" for k in range(srank.max() + 1)])
slot = hw & 0xF
print("end after the SIMD's first end, by wave slot:",
      [f"{k}: {erel[slot == k].mean():.2f}" for k in np.unique(slot)])
blk = np.nonzero(buf[:65536].view(-1, 8).cpu().numpy()[:, 0] > 0)[0] // 4
q = np.digitize(blk, np.percentile(blk, [25, 50, 75]))
print("end by block-index quartile (mean):", [f"{k}: {e_us[q == k].mean():.2f}" for k in range(4)])
print("corr(end - SIMD first end, fix steps):", np.corrcoef(erel, nfix)[0, 1])
# per-phase shader cycles (s_memtime) of each wave: segment setup (hypotheses,
# first loads), sub-chunk staging, hot loop, band fixes + the rest
ph = buf.cpu().numpy()[65536:65536 + 8 * 8192].reshape(-1, 8)[:len(t)].astype(np.float64)
if ph.sum() > 0:
    names = ["seg", "stage", "hot", "fix"]
    sub = ph[:, 4:7]
    print("fix parts per wave (median cycles): band re-check %d, exact flush %d, exact-only %d, rest (corrections, "
          "count atomics) %d" % (np.median(sub[:, 0]), np.median(sub[:, 1]), np.median(sub[:, 2]),
                                 np.median(ph[:, 3] - sub.sum(1))))
    ph = ph[:, :4]
    tot = ph.sum(1)
    print("phase cycles per wave (median):", {n: int(np.median(ph[:, k])) for k, n in enumerate(names)},
          "total", int(np.median(tot)))
    print("phase share of all wave cycles:", {n: round(float(ph[:, k].sum() / ph.sum()), 3) for k, n in enumerate(names)})
