"""Debug: the bench's latency graph (images one after another on one stream)
replayed a few times, for a rocprofv3 kernel trace of the sequential pipeline;
then `python tools/lat_trace.py --gaps <kernel_trace.csv>` prints each
kernel's median duration and the median idle gap before it.  GPU only; not
part of the product or the tests."""
import sys

import numpy as np

if len(sys.argv) > 2 and sys.argv[1] == "--gaps":
    import csv
    rows = list(csv.DictReader(open(sys.argv[2])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("<")[0])
                for r in rows)
    ev = [e for e in ev if e[2].startswith("k_")]
    dur, gap = {}, {}
    for i, (s, e, n) in enumerate(ev):
        dur.setdefault(n, []).append((e - s) / 1e3)
        if i:
            g = (s - ev[i - 1][1]) / 1e3
            if g < 50:                     # within a replay
                gap.setdefault(n, []).append(g)
    tot = 0.0
    for n in dur:
        d, g = np.median(dur[n]), np.median(gap.get(n, [0]))
        tot += d + g
        print(f"{n:18s} calls {len(dur[n]):5d}  median {d:7.2f} us  p10 {np.percentile(dur[n], 10):7.2f}"
              f"  gap before {g:6.2f} us")
    print(f"sum of medians + gaps per image: {tot:.2f} us")
    sys.exit(0)

import time  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, ".")
from pvnet_amd import ransac_voting_gpu as rvg, synth  # noqa: E402

NF, NLAT = 8, 32
segs, vers = [], []
for f in range(NF):
    fd = synth.synthetic_field(1234 + f)
    segs.append(torch.from_numpy(fd["seg"]).cuda())
    vers.append(torch.from_numpy(fd["vertex"]).cuda())
w = rvg.VotingWorkspace()
out = torch.zeros((NLAT, 9, 2), dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
for j in range(NLAT):                                # eager warm-up (workspace sizing)
    with torch.cuda.stream(s):
        rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], 512, _seed=3 + j, _workspace=w,
                                               out=out[j:j + 1])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for j in range(NLAT):
            rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], 512, _seed=3 + j, _workspace=w,
                                                   out=out[j:j + 1])
g.replay()
torch.cuda.synchronize()
R = int(sys.argv[1]) if len(sys.argv) > 1 else 10
t = time.perf_counter()
for _ in range(R):
    g.replay()
torch.cuda.synchronize()
print("latency us per image: %.2f" % ((time.perf_counter() - t) / (R * NLAT) * 1e6))
