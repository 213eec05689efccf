"""The voting half of configs[2] on the random-init network's own outputs
(fp16 batch 32, the bench's e2e setup): times v3 alone over the fixed
backbone outputs (one graph of the voting call, replayed), prints the
hypotheses' spread (how far the random field's line intersections land from
the image) and the per-kernel times when run under
`rocprofv3 --kernel-trace --stats -d DIR -o ev -- python3 tools/e2e_vote_probe.py`.
GPU only; not part of the product or the tests."""
import sys
import time

import torch

sys.path.insert(0, ".")
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402
from pvnet_amd.network import PVNet, PVNetInference  # noqa: E402

import os  # noqa: E402
import pvnet_amd.network as N  # noqa: E402
N.TAIL_SPLIT = os.environ.get("TAIL_SPLIT", "1") != "0"
print("tail split", N.TAIL_SPLIT)
torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
dev = torch.device("cuda")
B, H, W, VN = 32, 480, 640, 9
net = PVNetInference(PVNet(18, 2).eval()).to(dev).half().to(memory_format=torch.channels_last)
x = torch.randn(B, 3, H, W, device=dev).half().contiguous(memory_format=torch.channels_last)
with torch.no_grad():
    seg, ver = net(x)
torch.cuda.synchronize()
ws = rvg.VotingWorkspace()
out = torch.zeros((B, VN, 2), dtype=torch.float32, device=dev)
diag = {}
rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _workspace=ws, max_num=30000, _seed=7, _diag=diag)
torch.cuda.synchronize()
print("diag keys", sorted(diag))
if "hyp" in diag:
    h = diag["hyp"].float()
    r = torch.sqrt((h[..., 0] - W / 2) ** 2 + (h[..., 1] - H / 2) ** 2)
    for q in (0.5, 0.75, 0.9, 0.99):
        print(f"hypothesis distance from the image centre, q{q}: {torch.quantile(r.flatten()[:1000000], q).item():.1f} px")
print("tn", diag["tn"].cpu().tolist()[:8])


def once():
    return rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _workspace=ws, max_num=30000, _seed=7, out=out)


s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    for _ in range(3):
        once()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        once()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(30):
    g.replay()
torch.cuda.synchronize()
print(f"voting on the network's outputs, batch {B}: {(time.perf_counter() - t0) / 30 * 1e3:.4f} ms per batch")
