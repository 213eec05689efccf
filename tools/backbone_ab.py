"""A/B of the configs[2] backbone (fp16, batch 32, channels_last): the fused
inference form (PVNetInference.forward) against the module-epilogue form
(forward_modules), each captured in a hipGraph, interleaved rounds.
    python tools/backbone_ab.py [rounds] [which: both|fused|tail|modules] [batch]
(mio_tail: the fused form with convraw on MIOpen + pv_head instead of pv_decoder_tail)"""
import os
import sys
import time
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")   # as bench.py: no naive conv in Find
import torch
sys.path.insert(0, ".")
from pvnet_amd.network import PVNet, PVNetInference  # noqa: E402

torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
which = sys.argv[2] if len(sys.argv) > 2 else "both"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
dt = torch.float16 if B > 1 else torch.float32
net = PVNetInference(PVNet(18, 2).eval()).cuda().to(dt).to(memory_format=torch.channels_last)
x = torch.randn(B, 3, 480, 640).cuda().to(dt).contiguous(memory_format=torch.channels_last)


def graph(fn):
    s = torch.cuda.Stream()
    with torch.no_grad(), torch.cuda.stream(s):
        for _ in range(3):
            fn(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            fn(x)
    g.replay()
    torch.cuda.synchronize()
    return g


def forward_miopen_tail(x):
    net.fused_tail = False
    try:
        return net.forward(x)
    finally:
        net.fused_tail = True


gs = {}
if which in ("both", "fused"):
    gs["fused"] = graph(net.forward)
if which in ("both", "tail"):
    gs["mio_tail"] = graph(forward_miopen_tail)
if which in ("both", "modules"):
    gs["modules"] = graph(net.forward_modules)
for r in range(rounds):
    for k, g in gs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        dtm = (time.perf_counter() - t0) / 10
        print(f"round {r} {k:8s} {dtm * 1e3:.3f} ms/batch  {B / dtm:.1f} images/s  {144.9 * B / dtm / 1e3:.1f} TFLOP/s")
