"""Steady-state (hipGraph, back to back) time of the U1 call for the library
in PVVOTE_LIB (ablation variants: variants/u1nocomp.so, u1nostore.so)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from pvnet_amd import ransac_voting as rv  # noqa: E402
from pvnet_amd import synth  # noqa: E402
from tools.u1_graph_probe import graph_us, eager_us  # noqa: E402
from tools.u1_graph_probe import f, rows, cols, VN, hn  # noqa: E402

tn = 29861
coords = torch.from_numpy(np.stack([cols[:tn], rows[:tn]], 1).astype(np.float32)).cuda()
direct = torch.from_numpy(np.ascontiguousarray(
    f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows[:tn], cols[:tn]].transpose(2, 0, 1))).cuda()
idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
hyp = rv.generate_hypothesis(direct, coords, idxs)
inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
vote = lambda: rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)  # noqa: E731
import os  # noqa: E402
print(f"{os.environ.get('PVVOTE_LIB', 'product')}: graph {graph_us(vote):.1f} us, eager {eager_us(vote):.1f} us")
