"""Does the batch-1 stream gain when a frame's stages run on separate queues?
(A diagnostic, GPU only; not part of the product or the tests.)

    python tools/stream_pipeline_probe.py [steps] [nf,nv,nr,nws ...]

The headline stream (bench.run_stream) runs each frame's whole chain --
k_fg_count, k_compact (+ hypotheses), k_vote_mfma, k_refine_solve -- on one of
8 lane streams, so a lane's queue idles the matrix-core vote work while its
frame is in the latency-bound small kernels.  Here each frame is three calls
of the same ransac_voting_layer_v3_from_network, captured with
pv_debug_set_ablation so that each call keeps only its stage:

  front  (fg_count + compact + hypotheses)  on front stream  j % nf
  vote   (k_vote_mfma)                       on vote stream   j % nv, after front(j)
  refine (k_refine_solve -> keypoints)       on refine stream j % nr, after vote(j)

with a ring of nws workspaces (front(j) after refine(j - nws)).  Every frame's
keypoints are checked against its generating keypoints.  The plain 8-lane
stream runs first for reference."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import _lib  # noqa: E402
from pvnet_amd import ransac_voting_gpu as rvg  # noqa: E402

FRONT, VOTE, REFINE = 4 | 8, 1 | 16 | 8, 1 | 16 | 4


def pipelined(dev, segs, vers, kps, steps, nf, nv, nr, nws, M=int(os.environ.get("PROBE_M", "1024")), hn=512):
    L = _lib.load()
    L.pv_debug_set_ablation.argtypes = [ctypes.c_int32]
    NF = len(segs)
    works = [rvg.VotingWorkspace(check_streams=False) for _ in range(nws)]
    F = [bench.new_stream(dev) for _ in range(nf)]
    V = [bench.new_stream(dev) for _ in range(nv)]
    R = [bench.new_stream(dev) for _ in range(nr)]
    out = torch.zeros((M, 9, 2), dtype=torch.float32, device=dev)
    keep = []          # every event alive until the graph is instantiated

    def event():
        e = torch.cuda.Event()
        keep.append(e)
        return e

    dummy = [torch.zeros(1, device=dev) for _ in range(nws)]

    def call(j, seed, stage):
        if os.environ.get("PROBE_TRIVIAL"):      # the same DAG with one-element adds (runtime check)
            dummy[j % nws].add_(1.0)
            return
        L.pv_debug_set_ablation(stage)
        rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], hn, _seed=seed,
                                               _workspace=works[j % nws], out=out[j:j + 1])

    def body(seed0, staged):
        cur = torch.cuda.current_stream()
        for s in F + V + R:
            s.wait_stream(cur)
        ev_ref = [None] * nws
        for j in range(M):
            seed = seed0 + 17 * j
            fs, vs, rs = F[j % nf], V[j % nv], R[j % nr]
            if not staged:
                with torch.cuda.stream(fs):
                    if ev_ref[j % nws] is not None:
                        fs.wait_event(ev_ref[j % nws])
                    call(j, seed, 0)
                    e = event()
                    e.record(fs)
                    ev_ref[j % nws] = e
                continue
            with torch.cuda.stream(fs):
                if ev_ref[j % nws] is not None:
                    fs.wait_event(ev_ref[j % nws])
                call(j, seed, FRONT)
                e1 = event()
                e1.record(fs)
            with torch.cuda.stream(vs):
                vs.wait_event(e1)
                call(j, seed, VOTE)
                e2 = event()
                e2.record(vs)
            with torch.cuda.stream(rs):
                rs.wait_event(e2)
                call(j, seed, REFINE)
                e3 = event()
                e3.record(rs)
            ev_ref[j % nws] = e3
        L.pv_debug_set_ablation(0)
        for s in F + V + R:
            cur.wait_stream(s)

    cap = bench.new_stream(dev)
    with torch.cuda.stream(cap):
        for w in range(2):
            body(1000 * w, False)        # every workspace sized and holding a real frame
    torch.cuda.synchronize()
    g = bench.new_graph()
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            body(3, True)
    L.pv_debug_set_ablation(0)
    g.replay()
    torch.cuda.synchronize()
    err = float(np.abs(out.cpu().numpy() - kps[np.arange(M) % NF]).max())
    t0 = time.perf_counter()
    host = 0.0
    with torch.cuda.stream(cap):
        for _ in range(steps):
            h0 = time.perf_counter()
            g.replay()
            host += time.perf_counter() - h0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return steps * M / el, el / steps * 1e3, host / steps * 1e3, err


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfgs = [tuple(int(x) for x in c.split(",")) for c in sys.argv[2:]] or [(2, 4, 2, 16), (4, 4, 4, 16)]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    segs, vers, kps, tn = bench.make_fields(0, 1, 64, dev)
    args = argparse.Namespace(per_step=1024, inflight=8, warmup=3, hn=512)
    for rep in range(2):
        hs = {}
        if not os.environ.get("PROBE_SKIP_PLAIN"):
            el, local, _, _, _ = bench.run_stream(args, 1, 0, dev, segs, vers, steps, 0, stats=hs)
            err = float(np.abs(local.cpu().numpy() - kps[np.arange(steps * 1024) % 64]).max())
            print(f"plain 8 lanes: {steps * 1024 / el:.1f} images/s, {el / steps * 1e3:.3f} ms/step, host "
                  f"{hs['host_replay_s'] / steps * 1e3:.3f} ms/replay, max kp err {err:.3f}", flush=True)
        for nf, nv, nr, nws in cfgs:
            ips, ms, host, err = pipelined(dev, segs, vers, kps, steps, nf, nv, nr, nws)
            print(f"staged nf={nf} nv={nv} nr={nr} nws={nws}: {ips:.1f} images/s, {ms:.3f} ms/step, host "
                  f"{host:.3f} ms/replay, max kp err {err:.3f}", flush=True)


if __name__ == "__main__":
    main()
