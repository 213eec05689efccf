"""A/B of this round's backbone changes in one process, interleaved rounds:
fused downsample / two-map conv8s (PVNetInference.fused_ds) x the split-K
last round (network.CONV_SPLIT); fp16 batch 32, one hipGraph per variant,
timed by hipEvents.  GPU only; not part of the product or the tests."""
import sys

import torch

sys.path.insert(0, ".")
from pvnet_amd import network  # noqa: E402
from pvnet_amd.network import PVNet, PVNetInference  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda")
net = PVNetInference(PVNet(18, 2).eval()).to(dev).half().to(memory_format=torch.channels_last)
x = torch.randn(32, 3, 480, 640, device=dev).half().contiguous(memory_format=torch.channels_last)
variants = {"ds+split": (True, True), "ds": (True, False), "split": (False, True), "none": (False, False)}
graphs, outs = {}, {}
with torch.no_grad():
    for name, (ds, sp) in variants.items():
        net.fused_ds, network.CONV_SPLIT = ds, sp
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(2):
                net(x)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                outs[name] = net(x)
        graphs[name] = g
        g.replay()
    torch.cuda.synchronize()
    ref = outs["none"]
    for name in variants:
        d = max(float((a.float() - b.float()).abs().max()) for a, b in zip(outs[name], ref))
        print(f"{name:9s} max |out - none| {d:.3e}", flush=True)
    res = {k: [] for k in variants}
    for rnd in range(5):
        for name, g in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 5)
    for name, v in res.items():
        v = sorted(v)
        print(f"{name:9s} ms per forward: median {v[len(v) // 2]:.3f}  min {v[0]:.3f}  all {[round(t, 3) for t in v]}")
