"""Debug: the stem at configs[2]'s shape (fp16 batch 32, 480 x 640) timed by
events, 50 launches each: (a) pv_stem_conv_f16 then the pool-only maxpool
(two passes), (b) the fused pv_stem_pool_f16 when the library has it.  Run
per library variant (PVVOTE_LIB) for a same-box A/B.  GPU only."""
import sys

import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd.network import maxpool, stem_conv, stem_weights  # noqa: E402

# an older library variant without the fused entry point: bind the rest
_names = [s[0] for s in _lib.SIGNATURES]
import ctypes  # noqa: E402
_probe = ctypes.CDLL(_lib.LIB_PATH)
fused = hasattr(_probe, "pv_stem_pool_f16")
if not fused:
    _lib.SIGNATURES = [s for s in _lib.SIGNATURES if s[0] != "pv_stem_pool_f16"]

dev = torch.device("cuda:0")
cl = torch.channels_last
g = torch.Generator().manual_seed(5)
img = torch.randn(32, 3, 480, 640, generator=g).to(dev, torch.float16).contiguous(memory_format=cl)
c = torch.nn.Conv2d(3, 64, 7, 2, 3).to(dev)
with torch.no_grad():
    c.weight.copy_(torch.randn(64, 3, 7, 7, generator=g) * 0.1)
c = c.half()
w = stem_weights(c)


def timed(fn, k=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1000.0


with torch.no_grad():
    ta = timed(lambda: maxpool(stem_conv(img, w)))
    tc = timed(lambda: stem_conv(img, w))
    print(f"two passes: {ta:.1f} us (conv alone {tc:.1f} us)", flush=True)
    if fused:
        tb = timed(lambda: stem_conv(img, w, pool=True))
        x2, pl = stem_conv(img, w, pool=True)
        ok = torch.equal(pl, torch.nn.functional.max_pool2d(x2, 3, 2, 1))
        print(f"fused: {tb:.1f} us, pool equal: {ok}", flush=True)
