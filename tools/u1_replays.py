import sys, torch, numpy as np
sys.path.insert(0, ".")
import bench
from pvnet_amd import ransac_voting as rv, synth
dev = torch.device("cuda")
f = synth.synthetic_field(1234)
m = np.argmax(f["seg"][0], 0) == 1
rows, cols = np.nonzero(m)
coords = torch.from_numpy(np.stack([cols, rows], 1).astype(np.float32)).to(dev)
direct = torch.from_numpy(np.ascontiguousarray(f["vertex"][0].reshape(9, 2, 480, 640)[:, :, rows, cols].transpose(2, 0, 1))).to(dev)
tn = coords.shape[0]; hn = 512
idxs = torch.randint(0, tn, (hn, 9, 2), dtype=torch.int32, device=dev)
hyp = rv.generate_hypothesis(direct, coords, idxs)
inl = torch.empty((hn, 9, tn), dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(device=dev)
with torch.cuda.stream(s):
    for _ in range(5): rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for _ in range(100): rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
g.replay(); torch.cuda.synchronize()
for trial in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
    with torch.cuda.stream(s):
        ev[0].record(s)
        for k in range(6):
            g.replay(); ev[k + 1].record(s)
    torch.cuda.synchronize()
    print("trial", trial, [round(ev[k].elapsed_time(ev[k + 1]) * 10, 2) for k in range(6)], "us/launch")
