"""Host cost of the stream's graph launches, one thread: (a) one graph of
1,024 frames over 8 lanes (the bench's form), (b) one graph per lane (8
linear chains of 128 frames, each replayed on its own stream).  Reports the
host time inside the replay calls and the rate.  A diagnostic.
    python tools/lane_graphs_probe.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
NF, NL, PS, R = 64, 8, 1024, 20
segs, vers, kps, tn = bench.make_fields(0, 1, NF, dev)
works = [rvg.VotingWorkspace() for _ in range(NL)]
out = torch.zeros((PS, 9, 2), device=dev)


def vote(j, lane):
    rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], 512, _seed=j, _workspace=works[lane],
                                           out=out[j:j + 1])


# (a) one graph, 8 lanes forked from its stream
lanes = [bench.new_stream(dev) for _ in range(NL)]
cap = bench.new_stream(dev)


def body_a():
    for ln in lanes:
        ln.wait_stream(torch.cuda.current_stream())
    for j in range(PS):
        with torch.cuda.stream(lanes[j % NL]):
            vote(j, j % NL)
    for ln in lanes:
        torch.cuda.current_stream().wait_stream(ln)


with torch.cuda.stream(cap):
    body_a()
torch.cuda.synchronize()
ga = bench.new_graph()
with torch.cuda.stream(cap):
    with torch.cuda.graph(ga, stream=cap):
        body_a()
ga.replay()
torch.cuda.synchronize()
# (b) one linear graph per lane, each captured on its own stream
gb = []
for ln in range(NL):
    g = bench.new_graph()
    with torch.cuda.stream(lanes[ln]):
        with torch.cuda.graph(g, stream=lanes[ln]):
            for j in range(ln, PS, NL):
                vote(j, ln)
    gb.append(g)
for ln in range(NL):
    with torch.cuda.stream(lanes[ln]):
        gb[ln].replay()
torch.cuda.synchronize()
for trial in range(2):
    for name in ("a", "b"):
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for _ in range(R):
            if name == "a":
                with torch.cuda.stream(cap):
                    h0 = time.perf_counter()
                    ga.replay()
                    host += time.perf_counter() - h0
            else:
                for ln in range(NL):
                    with torch.cuda.stream(lanes[ln]):
                        h0 = time.perf_counter()
                        gb[ln].replay()
                        host += time.perf_counter() - h0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"form {name}: host in replay() {host * 1e3:.1f} ms, wall {dt * 1e3:.1f} ms -> {R * PS / dt:.0f} images/s",
              flush=True)
