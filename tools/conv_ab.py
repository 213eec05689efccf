"""A/B of k_conv3x3 builds on the backbone's wide 3x3 shapes (fp16,
channels_last, batch 32 at 60 x 80), one process per library so each loads
its own build, interleaved rounds; plus a hipBLASLt reference GEMM of
layer4's implicit-GEMM size (M 512, N 153,600, K 4,608) through torch.matmul.
GPU only; not part of the product or the tests.

    python tools/conv_ab.py ROUNDS LIB [LIB ...]      # driver
    python tools/conv_ab.py --one LIB                 # one library, one pass (child)
    python tools/conv_ab.py --gemm                    # the hipBLASLt reference
"""
import os
import subprocess
import sys
import time

SHAPES = ((128, 256, 2), (256, 256, 2), (256, 512, 4), (512, 512, 4), (512, 256, 1))


def graph(torch, fn, n=10):
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


def timed(torch, g, n=10, reps=5):
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * n) * 1e6


def one():
    import torch
    sys.path.insert(0, ".")
    from pvnet_amd.network import conv3x3
    torch.manual_seed(0)
    cl = torch.channels_last
    N, H, W = 32, 60, 80
    out = []
    for cin, cout, d in SHAPES:
        x = torch.randn(N, cin, H, W, device="cuda").half().contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)).half()
        b = torch.randn(cout, device="cuda").half()
        wk = w.permute(0, 2, 3, 1).contiguous()
        res = torch.randn(N, cout, H, W, device="cuda").half().contiguous(memory_format=cl)
        with torch.no_grad():
            y0 = conv3x3(x, wk, b, d, "relu", res=res).float().sum().item()
            g = graph(torch, lambda: conv3x3(x, wk, b, d, "relu", res=res))
            us = timed(torch, g)
        fl = 2 * cin * cout * 9 * N * H * W
        out.append(f"{cin}->{cout}d{d} {us:7.1f}us {fl / us / 1e6:6.1f}TF/s chk={y0:.6e}")
    print(" | ".join(out), flush=True)


def gemm():
    import torch
    torch.manual_seed(0)
    M, N, K = 512, 153600, 4608
    a = torch.randn(M, K, device="cuda").half()
    b = torch.randn(K, N, device="cuda").half()
    for name, fn in (("A[MxK] @ B[KxN]", lambda: a @ b),
                     ("B^T-major: (B^T[NxK] @ A^T) ", None)):
        if fn is None:
            bt = b.t().contiguous()
            at = a.t().contiguous()
            fn = lambda: bt @ at  # noqa: E731
        g = graph(torch, fn, n=5)
        for r in range(3):
            us = timed(torch, g, n=5)
            print(f"hipBLASLt fp16 {name} M={M} N={N} K={K}: {us:7.1f} us = {2 * M * N * K / us / 1e6:7.1f} TF/s "
                  f"({2 * M * N * K / us / 1e6 / 2500:.3f} of 2.5 PF)", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one()
    elif sys.argv[1] == "--gemm":
        gemm()
    else:
        rounds, libs = int(sys.argv[1]), sys.argv[2:]
        for r in range(rounds):
            for lib in libs:
                env = dict(os.environ, PVVOTE_LIB=lib)
                p = subprocess.run([sys.executable, __file__, "--one", lib], env=env, capture_output=True, text=True,
                                   timeout=300)
                if p.returncode != 0:
                    print(lib, "FAILED", p.returncode, p.stderr[-2000:], flush=True)
                    sys.exit(p.returncode)
                print(f"round {r} {os.path.basename(lib)}: {p.stdout.strip()}", flush=True)
