"""Per-layer device time of the configs[2] backbone (fp16, batch 32,
channels_last; LT_FORM=inference (default: PVNetInference) or folded): hipEvents around every leaf module and cat /
upsample in eager mode (after MIOpen's Find has run).  GPU only."""
import sys
import collections

import torch
from torch import nn

sys.path.insert(0, ".")
from pvnet_amd.network import PVNet, PVNetInference, fold_batchnorm  # noqa: E402

torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
import os
net = (PVNetInference(PVNet(18, 2).eval()) if os.environ.get("LT_FORM", "inference") == "inference"
       else fold_batchnorm(PVNet(18, 2).eval())).cuda().half().to(memory_format=torch.channels_last)
x = torch.randn(32, 3, 480, 640).cuda().half().contiguous(memory_format=torch.channels_last)
ev = collections.defaultdict(list)
pre = {}


def hook_pre(name):
    def f(m, inp):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        pre[name] = e
    return f


def hook_post(name):
    def f(m, inp, out):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev[name].append((pre[name], e, tuple(inp[0].shape), tuple(out.shape) if torch.is_tensor(out) else None))
    return f


for name, m in net.named_modules():
    if len(list(m.children())) == 0 and not isinstance(m, nn.Identity):
        m.register_forward_pre_hook(hook_pre(name))
        m.register_forward_hook(hook_post(name))
with torch.no_grad():
    for _ in range(3):
        net(x)
    torch.cuda.synchronize()
    ev.clear()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    net(x)
    b.record()
torch.cuda.synchronize()
tot = a.elapsed_time(b)
rows = []
for name, lst in ev.items():
    for s, e, ish, osh in lst:
        rows.append((s.elapsed_time(e), name, ish, osh))
acc = sum(r[0] for r in rows)
print(f"forward {tot:.3f} ms; leaf modules {acc:.3f} ms; rest (cat, slicing) {tot - acc:.3f} ms")
for t, name, ish, osh in sorted(rows, reverse=True)[:30]:
    print(f"{t:7.3f} ms  {name:32s} {ish} -> {osh}")
