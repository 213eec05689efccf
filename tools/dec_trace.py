"""Debug: per-phase stamps (s_memtime) of the warp-specialised decoder
convolutions (k_dec_conv: conv4s, then conv2s) at batch 32 -- consumer
phase time, its MFMA span and its wait for the weight DMA; producer loads,
build and patch writes -- medians over blocks and the first 4 tiles.
Needs a PVC_DEC_TRACE build:
    python tools/build_variant.py dectrace -DPVC_DEC_TRACE
    PVVOTE_LIB=variants/dectrace.so python tools/dec_trace.py
GPU only; not part of the product or the tests."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd import network as N  # noqa: E402

L = _lib.load()
L.pv_debug_set_dec_trace.argtypes = [ctypes.c_void_p]
cl = torch.channels_last
g = torch.Generator().manual_seed(3)
buf = torch.zeros(256 * 4 * 6 * 8, dtype=torch.int64, device="cuda")
for name, C1, CO, h, w in (("conv4s", 128, 64, 60, 80), ("conv2s", 64, 32, 120, 160)):
    fm = torch.randn(32, C1, h, w, generator=g).cuda().half().contiguous(memory_format=cl)
    skip = torch.randn(32, 64, 2 * h, 2 * w, generator=g).cuda().half().contiguous(memory_format=cl)
    c = torch.nn.Conv2d(C1 + 64, CO, 3, 1, 1).cuda().half()
    wts = N.decoder_conv4s_weights(c) if CO == 64 else N.decoder_conv2s_weights(c)
    fn = N.decoder_conv4s if CO == 64 else N.decoder_conv2s
    for _ in range(20):
        fn(fm, skip, wts, 0.1)
    buf.zero_()
    L.pv_debug_set_dec_trace(ctypes.c_void_p(buf.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn(fm, skip, wts, 0.1)
    e1.record()
    torch.cuda.synchronize()
    L.pv_debug_set_dec_trace(None)
    P = 6 if CO == 64 else 4
    t = buf.view(256, 4, 6, 8).cpu().numpy().astype(np.float64)[:, :, :P]
    ok = t[:, :, :, 0] > 0
    # phase length: consumer phase start to the next phase's start
    cs = t[:, :, :, 0]
    print(f"{name}: {e0.elapsed_time(e1) * 1e3:.1f} us; per phase (cycles of s_memtime, medians over blocks x tiles 1..3):")
    for j in range(P):
        sel = ok[:, 1:, j]
        d_mfma = (t[:, 1:, j, 1] - t[:, 1:, j, 0])[sel]
        d_wait = (t[:, 1:, j, 2] - t[:, 1:, j, 1])[sel]
        nxt = np.where(j + 1 < P, t[:, 1:, min(j + 1, P - 1), 0], np.roll(t[:, :, 0, 0], -1, axis=1)[:, 1:])
        d_phase = (nxt - t[:, 1:, j, 0])[sel & (nxt > 0)]
        # producer stamps: [4] phase start, [5] build done, [6] patch writes done, [7] loads issued
        p_build = (t[:, 1:, j, 5] - t[:, 1:, j, 4])[sel]
        p_write = (t[:, 1:, j, 6] - t[:, 1:, j, 5])[sel]
        p_load = (t[:, 1:, j, 7] - t[:, 1:, j, 6])[sel]
        p_arrive = (t[:, 1:, j, 7] - t[:, 1:, j, 0])[sel]
        print(f"  phase {j}: phase {np.median(d_phase):7.0f}  cons mfma {np.median(d_mfma):6.0f} wait {np.median(d_wait):6.0f}"
              f" | prod build {np.median(p_build):6.0f} patch writes {np.median(p_write):6.0f} loads {np.median(p_load):6.0f}"
              f" done@ {np.median(p_arrive):6.0f}", flush=True)
