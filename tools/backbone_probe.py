import time, torch, sys
sys.path.insert(0, '.')
from pvnet_amd.network import PVNet
torch.backends.cudnn.benchmark = True
dev = torch.device('cuda')
for half, dt_ in ((False, torch.float32), (True, torch.float16), (True, torch.bfloat16)):
    for cl in (True, False):
        torch.manual_seed(0)
        mf = torch.channels_last if cl else torch.contiguous_format
        net = PVNet(18, 2).to(dev).eval().to(dtype=dt_, memory_format=mf)
        x = torch.randn(1, 3, 480, 640, device=dev).to(dtype=dt_, memory_format=mf)
        with torch.no_grad():
            t0 = time.perf_counter()
            for _ in range(3): net(x)
            torch.cuda.synchronize(); tw = time.perf_counter() - t0
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    net(x)
            g.replay(); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20): g.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
        print(f"{str(dt_):15s} channels_last={cl}: {dt*1e3:.3f} ms  {144.9e9/dt/1e12:.1f} TFLOP/s (warmup {tw:.1f}s)", flush=True)
