"""k_conv3x3r (4-stage ring of 32-channel half steps) against k_conv3x3 (the
2-stage form it replaces): the same MFMA sequence, so pv_conv3x3_ex_f16's
outputs must be bit-identical.  Runs each case through the product library
and through an A/B build of the old form (variants/ring0.so: build with
    python tools/build_variant.py ring0 -DPVC_RING4=0
), one process.  GPU only; a check, not part of the tests."""
import sys

import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd import network as N  # noqa: E402

cl = torch.channels_last
g = torch.Generator().manual_seed(77)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, generator=g) * scale).cuda().half()


cases = []
# (name, x, w, bias, dil, stride, act, x2, mode2, s2, rbias)
x = rnd(8, 512, 60, 80).contiguous(memory_format=cl)
w = rnd(512, 3, 3, 512, scale=0.02).contiguous()
cases.append(("layer4 512->512 d4", x, w.reshape(512, -1).contiguous(), rnd(512), 4, 1, "relu", None, "none", 1, None))
x = rnd(8, 256, 60, 80).contiguous(memory_format=cl)
w = rnd(256, 3, 3, 256, scale=0.03).contiguous()
cases.append(("layer3 256->256 d2", x, w.reshape(256, -1).contiguous(), rnd(256), 2, 1, "relu", None, "none", 1, None))
x = rnd(8, 64, 120, 160).contiguous(memory_format=cl)
y = rnd(8, 128, 60, 80).contiguous(memory_format=cl)
w = torch.cat([rnd(128, 9 * 128, scale=0.03), rnd(128, 64, scale=0.1)], 1).contiguous()
cases.append(("layer2 conv2 + 1x1 ds s2", y, w, rnd(128), 1, 1, "relu", x, "1x1", 2, rnd(128)))
x = rnd(8, 64, 120, 160).contiguous(memory_format=cl)
w = rnd(128, 9 * 64, scale=0.05).contiguous()
cases.append(("layer2 conv1 s2", x, w, rnd(128), 1, 2, "relu", None, "none", 1, None))
x = rnd(8, 256, 60, 80).contiguous(memory_format=cl)
x2 = rnd(8, 128, 60, 80).contiguous(memory_format=cl)
w = rnd(256, 9 * 384, scale=0.02).contiguous()
cases.append(("conv8s cat 256+128", x, w, rnd(256), 1, 1, "leaky", x2, "cat", 1, None))


def run(path):
    _lib._lib = None
    _lib.LIB_PATH = path
    _lib.load()
    N.clear_conv_workspaces()
    outs = []
    with torch.no_grad():
        for name, x, w, b, d, st, act, x2, m2, s2, rb in cases:
            outs.append(N.conv3x3_ex(x, w, b, d, stride=st, act=act, x2=x2, mode2=m2, s2=s2, rbias=rb))
    torch.cuda.synchronize()
    return outs


new = run(_lib.os.path.join(_lib.HERE, "libpvvote.so"))
old = run("variants/ring0.so")
ok = True
for (name, *_), a, b in zip(cases, new, old):
    eq = torch.equal(a, b)
    ok &= eq
    print(f"{name}: bit-identical {eq}  max |diff| {float((a.float() - b.float()).abs().max()):.3e}", flush=True)
print("conv_ring_check", "ok" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
