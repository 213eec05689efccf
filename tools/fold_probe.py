"""Backbone forward time, BN folded vs not (fp16 batch 32 channels_last,
fp32 batch 1), each as a hipGraph of the forward.  GPU only."""
import sys
import time

import torch

sys.path.insert(0, ".")
from pvnet_amd.network import PVNet, fold_batchnorm  # noqa: E402

torch.backends.cudnn.benchmark = True


def timed(net, x, iters=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(3):
            net(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.no_grad(), torch.cuda.graph(g, stream=s):
        net(x)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


import os
CASES = ((True, 32),) if os.environ.get('FOLD_FP16_ONLY') else ((True, 32), (False, 1))
for half, b in CASES:
    dt = torch.float16 if half else torch.float32
    torch.manual_seed(0)
    base = PVNet(18, 2).eval()
    x = torch.randn(b, 3, 480, 640).cuda().to(dtype=dt, memory_format=torch.channels_last)
    for name, net in (("bn", base), ("folded", fold_batchnorm(base))):
        n = net.cuda().to(dtype=dt, memory_format=torch.channels_last)
        print(f"{'fp16' if half else 'fp32'} b{b} {name:7s} {timed(n, x):8.3f} ms", flush=True)
