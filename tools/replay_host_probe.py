"""Is the stream's graph launch host-bound?  One stream graph of 1,024
frames (bench.graph_stream's structure), then K replays timed twice: the
host time spent inside graph.replay() (submission) and the wall time to
the end of the GPU work.  A diagnostic, not part of the bench.
    python tools/replay_host_probe.py [per_step] [replays]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402

ps = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
NF, NL = 64, 8
segs, vers, kps, tn = bench.make_fields(0, 1, NF, dev)
works = [rvg.VotingWorkspace() for _ in range(NL)]
lanes = [bench.new_stream(dev) for _ in range(NL)]
out = torch.zeros((ps, 9, 2), device=dev)
cap = bench.new_stream(dev)


def body():
    for ln in lanes:
        ln.wait_stream(torch.cuda.current_stream())
    for j in range(ps):
        with torch.cuda.stream(lanes[j % NL]):
            rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], 512, _seed=j,
                                                   _workspace=works[j % NL], out=out[j:j + 1])
    for ln in lanes:
        torch.cuda.current_stream().wait_stream(ln)


with torch.cuda.stream(cap):
    body()
torch.cuda.synchronize()
g = bench.new_graph()
with torch.cuda.stream(cap):
    with torch.cuda.graph(g, stream=cap):
        body()
g.replay()
torch.cuda.synchronize()
for trial in range(3):
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    with torch.cuda.stream(cap):
        g.replay()
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    h2 = time.perf_counter()
    print(f"one replay on an idle device: host in replay() {1e3 * (h1 - h0):.2f} ms, to GPU end {1e3 * (h2 - h0):.2f} ms",
          flush=True)
    host = 0.0
    t0 = time.perf_counter()
    with torch.cuda.stream(cap):
        for _ in range(K):
            h0 = time.perf_counter()
            g.replay()
            host += time.perf_counter() - h0
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"per_step {ps}: {K} replays, host in replay() {host * 1e3:.2f} ms, submit loop {1e3 * (t1 - t0):.2f} ms, "
          f"wall to GPU end {1e3 * (t2 - t0):.2f} ms -> {K * ps / (t2 - t0):.0f} images/s", flush=True)
