"""MIOpen time of layer3/layer4-shaped convolutions (fp16, channels_last):
dilated on the full map vs dilation 1 on its d x d phase grids (space to
batch), each in a hipGraph of 10 launches.  GPU only."""
import os
import sys
import time
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
cl = torch.channels_last


def timeit(fn, n=10):
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
    t0 = time.perf_counter()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (3 * n) * 1e6


for cin, cout, d in ((256, 256, 2), (512, 512, 4), (256, 512, 4), (512, 256, 1)):
    N, H, W = 32, 60, 80
    x = torch.randn(N, cin, H, W, device="cuda").half().contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.02).half().contiguous(memory_format=cl)
    with torch.no_grad():
        t_dil = timeit(lambda: F.conv2d(x, w, None, 1, d, d))
        xp = x.view(N, cin, H // d, d, W // d, d).permute(0, 3, 5, 1, 2, 4).reshape(N * d * d, cin, H // d, W // d)
        xp = xp.contiguous(memory_format=cl)
        t_ph = timeit(lambda: F.conv2d(xp, w, None, 1, 1, 1))
        # exactness of the phase form
        y = F.conv2d(x, w, None, 1, d, d)
        yp = F.conv2d(xp, w, None, 1, 1, 1).reshape(N, d, d, cout, H // d, W // d).permute(0, 3, 4, 1, 5, 2)
        yp = yp.reshape(N, cout, H, W)
        err = (y.float() - yp.float()).abs().max().item()
    fl = 2 * cin * cout * 9 * N * H * W
    print(f"cin {cin} cout {cout} d {d}: dilated {t_dil:7.1f} us ({fl / t_dil / 1e6:6.1f} TF/s), "
          f"phase grids {t_ph:7.1f} us ({fl / t_ph / 1e6:6.1f} TF/s), max |diff| {err:.3e}", flush=True)
