"""Per-kernel breakdown of the configs[2] backbone (fp16, batch 32,
channels-last PVNetInference): run it under
`rocprofv3 --kernel-trace --stats -d DIR -o bb -- python3 tools/bb_kernels.py`
(10 graph replays after a warm-up), then
`python3 tools/bb_kernels.py --summary DIR/bb_kernel_trace.csv` prints each
kernel's time per forward over the last REPS replays.  GPU only; not part of the product or the tests."""
import csv
import sys

REPS = 10

if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    K = next(k for k in range(1, len(names) // 2) if names[-k:] == names[-2 * k:-k])   # kernels per forward
    last = rows[-REPS * K:]
    per = {}
    for i, r in enumerate(last):
        key = (i % K, r["Kernel_Name"][:100])
        per[key] = per.get(key, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / REPS
    span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3 / REPS
    for (i, name), us in sorted(per.items()):
        print(f"{i:3d} {us:9.1f} us  {name}")
    print(f"{K} kernels per forward, sum {sum(per.values()):.1f} us, wall {span:.1f} us per forward")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, ".")
from pvnet_amd.network import PVNet, PVNetInference  # noqa: E402

import os  # noqa: E402
import pvnet_amd.network as N  # noqa: E402
N.TAIL_SPLIT = os.environ.get("TAIL_SPLIT", "1") != "0"
torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
dev = torch.device("cuda")
net = PVNetInference(PVNet(18, 2).eval()).to(dev).half().to(memory_format=torch.channels_last)
x = torch.randn(32, 3, 480, 640, device=dev).half().contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    for _ in range(3):          # MIOpen Find + weight layouts (excluded: profile starts after?)
        net(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            net(x)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"backbone fp16 batch 32: {e0.elapsed_time(e1) / REPS:.3f} ms per forward", flush=True)
