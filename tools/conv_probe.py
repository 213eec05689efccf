"""pv_conv3x3_f16 against MIOpen (+ the HIP epilogue) on the backbone's wide
3x3 shapes (fp16, channels_last, batch 32 at 60 x 80), each in a hipGraph of
10 launches, interleaved rounds.  GPU only.
    python tools/conv_probe.py [rounds]"""
import os
import sys
import time
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from pvnet_amd.network import conv3x3, conv_epilogue  # noqa: E402

torch.backends.cudnn.benchmark = True
cl = torch.channels_last


def graph(fn, n=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    return g


def timed(g, n=10, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * n) * 1e6


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
N, H, W = 32, 60, 80
for cin, cout, d in ((128, 256, 2), (256, 256, 2), (256, 512, 4), (512, 512, 4), (512, 256, 1)):
    x = torch.randn(N, cin, H, W, device="cuda").half().contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).half()
    b = torch.randn(cout, device="cuda").half()
    wk = w.permute(0, 2, 3, 1).contiguous()
    res = torch.randn(N, cout, H, W, device="cuda").half().contiguous(memory_format=cl)
    with torch.no_grad():
        gm = graph(lambda: conv_epilogue(F.conv2d(x, w, None, 1, d, d), b, "relu", res=res))
        gh = graph(lambda: conv3x3(x, wk, b, d, "relu", res=res))
        for r in range(rounds):
            tm, th = timed(gm), timed(gh)
            fl = 2 * cin * cout * 9 * N * H * W
            print(f"{cin}->{cout} d{d} round {r}: MIOpen+epilogue {tm:7.1f} us ({fl / tm / 1e6:6.1f} TF/s)  "
                  f"pv_conv3x3 {th:7.1f} us ({fl / th / 1e6:6.1f} TF/s)", flush=True)
