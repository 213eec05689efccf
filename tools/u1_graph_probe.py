"""voting_for_hypothesis (dense bytes) launched back to back in a hipGraph
(the steady state, every launch's writes draining to HBM behind the next)
against eager launches with events between them, for row lengths tn that are
and are not multiples of 128 bytes, beside fill_ of the same bytes.  GPU only."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import ransac_voting as rv  # noqa: E402
from pvnet_amd import synth  # noqa: E402

f = synth.synthetic_field(1234)
m = np.argmax(f["seg"][0], 0) == 1
rows, cols = np.nonzero(m)
VN, hn = 9, 512


def graph_us(fn, reps=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a.record(s)
        g.replay()
        b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def eager_us(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for x, y in ev:
        x.record()
        fn()
        y.record()
    torch.cuda.synchronize()
    return float(np.median([x.elapsed_time(y) for x, y in ev])) * 1e3


def main():
  for tn in (29861, 29824, 29696):
      coords = torch.from_numpy(np.stack([cols[:tn], rows[:tn]], 1).astype(np.float32)).cuda()
      direct = torch.from_numpy(np.ascontiguousarray(
          f["vertex"][0].reshape(VN, 2, 480, 640)[:, :, rows[:tn], cols[:tn]].transpose(2, 0, 1))).cuda()
      idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device="cuda")
      hyp = rv.generate_hypothesis(direct, coords, idxs)
      inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device="cuda")
      vote = lambda: rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)  # noqa: E731
      fill = lambda: inl.fill_(1)  # noqa: E731
      n = inl.numel()
      gv, ev_, gf, ef = graph_us(vote), eager_us(vote), graph_us(fill), eager_us(fill)
      print(f"tn={tn} (mod 128 = {tn % 128}): vote graph {gv:.1f} us ({n / gv / 1e3:.0f} GB/s)  eager {ev_:.1f} us | "
            f"fill_ graph {gf:.1f} us ({n / gf / 1e3:.0f} GB/s)  eager {ef:.1f} us")
  big = torch.empty(2 * 137_599_488, dtype=torch.uint8, device="cuda")
  for nb in (137_599_488, 2 * 137_599_488):
      x = big[:nb]
      g = graph_us(lambda: x.fill_(1))
      print(f"fill_ {nb / 1e6:.0f} MB graph {g:.1f} us = {nb / g / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
