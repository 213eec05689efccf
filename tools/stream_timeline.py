"""Where the batch-1 headline stream's time goes (a diagnostic, GPU only).

    python tools/stream_timeline.py run [steps]          # the headline stream (bench.run_stream), plain
    python tools/stream_timeline.py empty [steps]        # the same graph shape, n trivial kernels per frame
    python tools/stream_timeline.py --analyze trace.csv  # a rocprofv3 kernel trace of `run`
    python tools/stream_timeline.py abl [steps] m1,m2,..  # `run` with pipeline kernels left out of the graph

`abl` warms every lane up with the whole pipeline (so each lane's workspace
holds a real frame's records, hypotheses and pixel count), then captures the
graph with the kernels of mask m left out (pv_debug_set_ablation: 1 k_compact,
2 k_hyp_gen, 4 vote, 8 refine, 16 k_fg_count): what the stream costs without
them, on real data.

`empty` replays graphs of the headline's shape (1,024 frames per replay, 8
lanes forked from the capture stream and joined) whose frames are n = 1..5
one-element fills instead of the v3 chain: the host time inside
graph.replay() and the wall time per replay then are the runtime's
submission and the command processor's dispatch alone, the floor under any
number of kernel nodes per frame.

`--analyze` takes the last replays of the trace and reports the fraction of
time at least one kernel ran (GPU busy), the mean number of kernels running,
and per queue the idle gap between a kernel's end and the next kernel's start."""
import sys
import time

import numpy as np


def analyze(path, last_ms=60.0):
    import csv
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].split("<")[0].replace("(anonymous namespace)::", ""),
                 r.get("Queue_Id", "?")) for r in rows)
    ev = [e for e in ev if e[2].startswith("k_")]
    t_end = max(e[1] for e in ev)
    ev = [e for e in ev if e[0] >= t_end - last_ms * 1e6]
    t0 = min(e[0] for e in ev)
    span = t_end - t0
    # union of intervals and time-weighted concurrency
    pts = sorted([(e[0], 1) for e in ev] + [(e[1], -1) for e in ev])
    busy, conc, cur, last = 0, 0.0, 0, pts[0][0]
    hist = {}
    for t, d in pts:
        dt = t - last
        if cur > 0:
            busy += dt
        conc += cur * dt
        hist[cur] = hist.get(cur, 0) + dt
        cur += d
        last = t
    print(f"window {span / 1e6:.2f} ms, {len(ev)} kernels, busy {busy / span:.3f}, mean running {conc / span:.2f}")
    print("time share by kernels running:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
    byq = {}
    for e in ev:
        byq.setdefault(e[3], []).append(e)
    for q, es in sorted(byq.items()):
        es.sort()
        gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(es, es[1:])]
        g = np.array(gaps)
        print(f"queue {q}: {len(es)} kernels, gap median {np.median(g):.2f} us p10 {np.percentile(g, 10):.2f} "
              f"p90 {np.percentile(g, 90):.2f}, busy {sum(e[1] - e[0] for e in es) / span:.3f}")
    names = sorted({e[2] for e in ev})
    for n in names:
        d = np.array([(e[1] - e[0]) / 1e3 for e in ev if e[2] == n])
        print(f"{n:18s} {len(d):6d} launches, median {np.median(d):6.2f} us, sum/window {d.sum() * 1e3 / span:.3f}")


def main():
    if sys.argv[1] == "--analyze":
        return analyze(sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 60.0)
    import argparse
    import torch
    sys.path.insert(0, ".")
    import bench
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    args = argparse.Namespace(per_step=1024, inflight=8, warmup=3, hn=512)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    if sys.argv[1] == "abl":
        import ctypes
        from pvnet_amd import _lib
        L = _lib.load()
        L.pv_debug_set_ablation.argtypes = [ctypes.c_int32]
        segs, vers, kps, tn = bench.make_fields(0, 1, 64, dev)
        orig = bench.new_graph
        for m in [int(x) for x in sys.argv[3].split(",")]:
            def ng(m=m):
                L.pv_debug_set_ablation(m)
                return orig()
            bench.new_graph = ng
            hs = {}
            el, _, _, _, _ = bench.run_stream(args, 1, 0, dev, segs, vers, steps, 0, stats=hs)
            L.pv_debug_set_ablation(0)
            bench.new_graph = orig
            print(f"abl {m:2d}: {steps * 1024 / el:.1f} images/s, {el / steps * 1e3:.3f} ms/step, host "
                  f"{hs['host_replay_s'] / steps * 1e3:.3f} ms/replay", flush=True)
        return
    if sys.argv[1] == "run":
        segs, vers, kps, tn = bench.make_fields(0, 1, 64, dev)
        hs = {}
        el, local, _, _, _ = bench.run_stream(args, 1, 0, dev, segs, vers, steps, 0, stats=hs)
        err = float(np.abs(local.cpu().numpy() - kps[np.arange(steps * 1024) % 64]).max())
        print(f"run: {steps * 1024 / el:.1f} images/s, {el / steps * 1e3:.3f} ms/step, host "
              f"{hs['host_replay_s'] / steps * 1e3:.3f} ms/replay, max kp err {err:.3f}", flush=True)
        return
    dummies = [torch.zeros(1, device=dev) for _ in range(8)]
    for n in (1, 2, 3, 4, 5):
        def vote(j, seed, lane, outs, n=n):
            for _ in range(n):
                dummies[lane].add_(1.0)
        hs = {}
        t = time.perf_counter()
        el, _, _, _ = bench.graph_stream(args, 1, 0, dev, steps, 0, vote, [((1,), torch.float32)], stats=hs)
        print(f"empty n={n}: {el / steps * 1e3:.3f} ms/replay (= {steps * 1024 / el:.0f} frames/s), host "
              f"{hs['host_replay_s'] / steps * 1e3:.3f} ms/replay, {hs['host_replay_s'] / steps / (1024 * n) * 1e6:.2f}"
              f" us/node", flush=True)


if __name__ == "__main__":
    main()
