"""Phase stamps of k_decoder_tail (PVT_TRACE build: variants/tail_trace.so):
per (block, tile iteration, wave) s_memtime at 8 points of the tile loop.
    PVVOTE_LIB=variants/tail_trace.so python tools/tail_trace.py"""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd.network import decoder_tail, decoder_tail_weights  # noqa: E402

cl = torch.channels_last
torch.manual_seed(0)
n, h, w = 32, 240, 320
fm = torch.randn(n, 32, h, w, device="cuda").half().contiguous(memory_format=cl)
img = torch.randn(n, 3, 2 * h, 2 * w, device="cuda").half().contiguous(memory_format=cl)
c0 = torch.nn.Conv2d(35, 32, 3, 1, 1).cuda().half()
c1 = torch.nn.Conv2d(32, 20, 1).cuda().half()
wts = decoder_tail_weights(c0, c1)
lib = _lib.load()
fn = lib.pv_debug_set_tail_trace
fn.argtypes = [ctypes.c_void_p]
nblk = 1024                                              # >= the grid (PVT_WPE blocks per CU)
tr = torch.zeros(nblk * 8 * 4 * 8, dtype=torch.int64, device="cuda")
for _ in range(3):
    decoder_tail(fm, img, wts)
fn(tr.data_ptr())
decoder_tail(fm, img, wts)
torch.cuda.synchronize()
fn(None)
t = tr.cpu().numpy().reshape(nblk, 8, 4, 8).astype(np.float64)
t = t[(t[:, 6, :, 7] > 0).all(axis=1)]                   # blocks of the grid with >= 7 tiles
# round 4 layout: 0 top, 1 after the wait for the fetch, 2 after barrier 1,
# (3, 4 = 2), 5 after the halo build, 6 after barrier 2, 7 after fetch + conv
names = ["wait fetch (vmcnt)", "barrier1", "-", "-", "halo build", "barrier2",
         "fetch+conv", "epilogue->next top"]
d = np.diff(t, axis=3)                                   # phases 0..6
nxt = t[:, 1:, :, 0] - t[:, :-1, :, 7]                   # epilogue (+loop) to next tile's top
tot = t[:, 1:, :, 0] - t[:, :-1, :, 0]
print("median cycles per phase (iterations 1..6, all waves):")
for k in range(7):
    print(f"  {names[k]:20s} {np.median(d[:, 1:7, :, k]):8.0f}   p90 {np.percentile(d[:, 1:7, :, k], 90):8.0f}")
print(f"  {names[7]:20s} {np.median(nxt[:, 1:6]):8.0f}   p90 {np.percentile(nxt[:, 1:6], 90):8.0f}")
print(f"  tile total           {np.median(tot[:, 1:6]):8.0f}   p90 {np.percentile(tot[:, 1:6], 90):8.0f}")
