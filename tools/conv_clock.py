"""In-kernel shader clock of k_conv3x3 on the backbone's wide shapes (fp16,
batch 32, 60 x 80): >= 2 s of back-to-back launches, then one launch whose
blocks stamp s_memtime / s_memrealtime around their K loop; clock =
d(memtime) / d(memrealtime) x 100 MHz, median over blocks (MI355X_MICROARCH
"DVFS give-back", item 6).  Needs a PVC_CLOCK_TRACE build:
    python tools/build_variant.py convclk -DPVC_CLOCK_TRACE
    PVVOTE_LIB=variants/convclk.so python tools/conv_clock.py
GPU only; a diagnostic, not part of the product or the tests."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd.network import conv3x3  # noqa: E402

L = _lib.load()
L.pv_debug_set_conv_clk.argtypes = [ctypes.c_void_p]
cl = torch.channels_last
N, H, W = 32, 60, 80
buf = torch.zeros(4 * 4096, dtype=torch.int64, device="cuda")
for cin, cout, d in ((256, 256, 2), (512, 512, 4)):
    x = torch.randn(N, cin, H, W, device="cuda").half().contiguous(memory_format=cl)
    wk = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).half().permute(0, 2, 3, 1).contiguous()
    b = torch.randn(cout, device="cuda").half()
    with torch.no_grad():
        for _ in range(3):
            conv3x3(x, wk, b, d, "relu")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        while time.perf_counter() - t0 < 2.5:
            for _ in range(20):
                conv3x3(x, wk, b, d, "relu")
            n += 20
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        buf.zero_()
        L.pv_debug_set_conv_clk(ctypes.c_void_p(buf.data_ptr()))
        conv3x3(x, wk, b, d, "relu")
        torch.cuda.synchronize()
        L.pv_debug_set_conv_clk(None)
    t = buf.view(-1, 4).cpu().numpy().astype(np.float64)
    t = t[t[:, 1] > 0]
    ghz = (t[:, 2] - t[:, 0]) / ((t[:, 3] - t[:, 1]) * 10.0)       # memrealtime ticks at 100 MHz = 10 ns
    fl = 2 * cin * cout * 9 * N * H * W
    tf = fl / us / 1e6
    clk = float(np.median(ghz))
    peak_at = 2500.0 * clk / 2.4
    print(f"{cin}->{cout} d{d}: {us:7.1f} us per launch ({tf:6.1f} TF/s = {tf / 2500:.3f} of 2.5 PF); in-kernel clock "
          f"median {clk:.3f} GHz (p10 {np.percentile(ghz, 10):.3f}, p90 {np.percentile(ghz, 90):.3f}; {len(ghz)} blocks) "
          f"-> dense peak at that clock {peak_at:.0f} TF/s, {tf / peak_at:.3f} of it", flush=True)
