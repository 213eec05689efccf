"""Diagnostic: one bench stream graph of `per_step` frames (8 lanes, so
per_step / 8 x 5 dependent kernels per lane) captured, uploaded and
replayed -- does a deep lane chain crash the graph launch?
    python tools/deep_graph_probe.py PER_STEP"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402

ps = int(sys.argv[1])
args = argparse.Namespace(per_step=ps, inflight=8, warmup=1, hn=512)
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
NF = 64
segs, vers, kps, tn = bench.make_fields(0, 1, NF, dev)
works = [rvg.VotingWorkspace() for _ in range(args.inflight)]


def vote(j, seed, lane, outs):
    rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], args.hn, _seed=seed,
                                           _workspace=works[lane], out=outs[0][j:j + 1])


el, local, allr, s = bench.graph_stream(args, 1, 0, dev, 2, 0, vote, [((9, 2), torch.float32)])
print("per_step", ps, "lane depth", ps // 8 * 5, "kernels; images/s", round(2 * ps / el, 1), flush=True)
