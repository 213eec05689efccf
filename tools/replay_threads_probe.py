"""Two host threads submitting the bench's stream graphs at once.

Each thread owns everything its graph touches: 8 lane streams and a capture
stream (pvnet_amd.streams.new_stream -- real streams, not torch's pool of
32), 8 VotingWorkspaces, its output rows; every thread's graph votes
`per_step` frames (bench.graph_stream's structure: frames alternate over the
lanes).  Graphs are captured one at a time (a capture in global mode must not
overlap another thread's work), then every thread replays its own graph
`replays` times at once.  Reports images/s for 1 and 2 threads, and checks
that every replay's keypoints equal the single-thread replay's, bit for bit.

Round 4's version of this probe (not committed) faulted with two threads
(hipErrorIllegalAddress in replay); DESIGN.md section 2a has the cause (its
threads' graphs shared one set of workspaces; the kernels then trusted the
pixel counts they read back).  A diagnostic, not part of the bench:
    python tools/replay_threads_probe.py [per_step] [replays] [shared]
With `shared` the run ends with the caller error round 4's probe most likely
made: two threads' graphs captured with ONE set of workspaces and output rows,
replayed at once -- the library must not fault (every kernel bounds the pixel
counts it reads from the workspace); the keypoints may come out wrong."""
import sys
import threading
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402
from pvnet_amd import streams  # noqa: E402

ps = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
SHARED = len(sys.argv) > 3 and sys.argv[3] == "shared"
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
NF, NL = 64, 8
segs, vers, kps, tn = bench.make_fields(0, 1, NF, dev)


class Lane:
    """One thread's graph: its own lanes, capture stream, workspaces, outputs."""

    def __init__(self, share=None):
        self.lanes = [streams.new_stream(dev) for _ in range(NL)]
        self.cap = streams.new_stream(dev)
        self.works = [rvg.VotingWorkspace() for _ in range(NL)] if share is None else share.works
        self.out = torch.zeros((ps, 9, 2), device=dev) if share is None else share.out

    def body(self):
        cur = torch.cuda.current_stream()
        for ln in self.lanes:
            ln.wait_stream(cur)
        for j in range(ps):
            with torch.cuda.stream(self.lanes[j % NL]):
                rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], 512, _seed=j,
                                                       _workspace=self.works[j % NL], out=self.out[j:j + 1])
        for ln in self.lanes:
            cur.wait_stream(ln)

    def capture(self):
        with torch.cuda.stream(self.cap):
            self.body()                      # eager warm-up: workspaces sized
        torch.cuda.synchronize()
        self.g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.cap):
            with torch.cuda.graph(self.g, stream=self.cap):
                self.body()
        self.g.replay()
        torch.cuda.synchronize()


def run(nthreads, ref=None, shared=False):
    ls = [Lane() for _ in range(nthreads)]
    if shared:
        ls = ls[:1] + [Lane(share=ls[0]) for _ in range(nthreads - 1)]
    for ln in ls:                             # one capture at a time
        ln.capture()
    if ref is not None and not shared:
        for ln in ls:
            assert torch.equal(ln.out, ref), "captured replay differs from the single-thread result"
    go = threading.Barrier(nthreads + 1)
    errs, bad = [], []

    def work(ln):
        try:
            torch.cuda.set_device(0)
            go.wait()
            with torch.cuda.stream(ln.cap):
                for _ in range(K):
                    ln.g.replay()
            ln.cap.synchronize()
            if ref is not None and not torch.equal(ln.out, ref):
                bad.append(1)
        except BaseException as e:            # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=work, args=(ln,)) for ln in ls]
    for t in th:
        t.start()
    torch.cuda.synchronize()
    go.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    if errs:
        raise errs[0]
    print(f"threads {nthreads}{' SHARED workspaces/outputs' if shared else ''}: {K} replays each of {ps} frames -> "
          f"{nthreads * K * ps / dt:.0f} images/s, outputs equal to the single-thread run: {not bad}", flush=True)
    assert shared or not bad
    return ls[0].out.clone()


ref = run(1)
run(1, ref)
run(2, ref)
run(2, ref)
if SHARED:
    run(2, ref, shared=True)
    torch.cuda.synchronize()
    print("shared run ended without a fault", flush=True)
print("replay_threads_probe ok", flush=True)
