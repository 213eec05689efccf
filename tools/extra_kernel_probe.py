"""How much one more kernel launch per frame costs the stream: the bench's
graph-replayed lanes (bench.graph_stream) voting the same resident fields,
with 0 / 1 / 2 tiny extra kernels (a 1-element add) after each frame's v3
call on its lane.  Interleaved rounds; a diagnostic, not part of the bench.
    python tools/extra_kernel_probe.py [rounds] [pool]
Each round captures, replays and drops three bench-size graphs (12 over 4
rounds: the graph churn behind round 4's keep-alive question).  `pool` takes
the lanes from torch.cuda.Stream() (round 4's bench: a pool of 32 streams per
priority, reused after 3.5 graph_stream calls) instead of new streams."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
if len(sys.argv) > 2 and sys.argv[2] == "pool":
    bench.new_stream = lambda dev: torch.cuda.Stream(device=dev)
args = argparse.Namespace(per_step=1024, inflight=8, warmup=3, hn=512)
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
NF = 64
segs, vers, kps, tn = bench.make_fields(0, 1, NF, dev)
works = [rvg.VotingWorkspace() for _ in range(args.inflight)]
dummies = [torch.zeros(1, device=dev) for _ in range(args.inflight)]
for r in range(rounds):
    for extra in (0, 1, 2):
        def vote(j, seed, lane, outs, extra=extra):
            rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], args.hn, _seed=seed,
                                                   _workspace=works[lane], out=outs[0][j:j + 1])
            for _ in range(extra):
                dummies[lane].add_(1.0)
        el, local, allr, s = bench.graph_stream(args, 1, 0, dev, 10, 0, vote, [((9, 2), torch.float32)])
        print("round", r, "extra kernels per frame", extra, "images/s", round(10 * args.per_step / el, 1), flush=True)
