"""Benchmark: images/sec of PVNet's vote -> keypoint hot path on MI355X.

The stream: synthetic 480x640, 9-keypoint batch-1 frames (generator S(seed),
~30k foreground pixels), 64 distinct fields per GPU resident
in HBM and cycled, each pushed through ``ransac_voting_layer_v3`` in its
fused network-layout form (seg_pred argmax + compaction + 512
hypotheses/keypoint + vote/count + LS refine).  One step = one replay of a
hipGraph voting --per-step frames (default 128) with 8 in flight on separate
streams.  Multi-GPU: one process per GPU, the stream's images sharded
round-robin (pvnet_amd.distributed.shard: weak scaling), one RCCL all_gather
of every image's keypoints in stream order (gather_results) at the end of
the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--per-step M]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset) the process
starts the N ranks itself (launch_ranks: one child per GPU carrying RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_*, before this process makes any GPU call).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# MIOpen's Find (cudnn.benchmark) also times its naive reference convolution,
# which is never the fastest: ~34 s of GPU time per bench run went to it
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level table)
HBM_PEAK_GBS = 8000.0
FP32_VECTOR_PEAK_TFLOPS = 157.3
H, W, VN = 480, 640, 9


PMC_FILE = "profiles/r06_pmc_traffic.json"
U1_WARM, U1_TIMED = 5, 3            # measure_u1: graph replays (of 100 launches) untimed, then timed
STATS_FILE = "profiles/r06_bench_kernel_stats.csv"


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (PMC_FILE: 2*FETCH_SIZE + WRITE_SIZE, collected with tools/pmc_traffic.sh
    on the bench command), or None."""
    try:
        with open(os.path.join(REPO, PMC_FILE)) as f:
            return json.load(f)["kernels"][kernel]["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


_STREAMS = []


def new_stream(dev):
    """A HIP stream of its own (pvnet_amd.streams.new_stream: torch.cuda.Stream()
    hands out one of a pool of 32 per priority, round robin, so the bench's
    ~40 lanes and capture streams would wrap onto each other's); like torch's
    pooled streams it lives for the whole process."""
    from pvnet_amd import streams
    st = streams.new_stream(dev)
    _STREAMS.append(st)
    return st


_GRAPHS = []


def new_graph():
    """A hipGraph kept alive for the whole process (with the streams it was
    captured on): round 5's host SIGSEGV in a variant build's bench run has
    no surviving record, so no graph is destroyed while the
    process runs."""
    g = torch.cuda.CUDAGraph()
    _GRAPHS.append(g)
    return g


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--per-step", type=int, default=1024,
                    help="images per GPU per step: one step = one replay of a hipGraph that votes this many "
                         "batch-1 frames (configs[1]), `--inflight` of them at a time on separate streams (the "
                         "graph's fork and join cost ~0.17 ms per replay: 128 frames per step 49.2k images/s, "
                         "512 51k, 1024 51.6k, 2048 52.3k on one box; DESIGN.md 7)")
    ap.add_argument("--fields", type=int, default=64,
                    help="distinct resident S(seed) fields per GPU the stream cycles through (64 x 24.6 MB: the "
                         "~5 MB each image reads, x64, exceeds the 256 MiB Infinity Cache, so inputs come from HBM)")
    ap.add_argument("--hn", type=int, default=512, help="round_hyp_num (DEMO:55 / TRAIN:141)")
    ap.add_argument("--inflight", type=int, default=8,
                    help="images in flight: consecutive images alternate over this many HIP streams (own workspaces)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--skip-e2e", action="store_true")
    ap.add_argument("--skip-u1", action="store_true")
    ap.add_argument("--skip-config3", action="store_true", help="skip the configs[3] and configs[4] stream legs")
    ap.add_argument("--skip-u4", action="store_true", help="skip the U4 (EVD with mean) timing")
    ap.add_argument("--skip-batched", action="store_true", help="skip the stream_batched4 leg")
    ap.add_argument("--share-device", action="store_true",
                    help="test hook for a one-GPU box: every rank on cuda:0 over gloo (RCCL refuses two ranks on one "
                         "device), the real GPU path otherwise -- checks the N > 1 code, not its speed")
    ap.add_argument("--dry-run", action="store_true",
                    help="the multi-rank plumbing without a GPU (CPU tests): gloo ranks, each image's result is its "
                         "field's generating keypoints (no voting), then the timed region's barriers, the gather, "
                         "the max over ranks and the stream-order check of a real run; the line says dry_run")
    return ap.parse_args()


def visible_gpus():
    """GPUs this process would see, without any HIP call: the KFD topology
    nodes with SIMDs (/sys/class/kfd/kfd/topology/nodes/*/properties), cut
    by ROCR_/HIP_/CUDA_VISIBLE_DEVICES when set; None if sysfs is unreadable
    (the ranks then check for themselves, setup_dist)."""
    import glob
    try:
        n = 0
        for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(p) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            n += int(props.get("simd_count", "0")) > 0
    except (OSError, ValueError):
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def _parse_cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def _fmt_cpulist(cpus):
    cpus, runs = sorted(cpus), []
    for c in cpus:
        if runs and c == runs[-1][1] + 1:
            runs[-1][1] = c
        else:
            runs.append([c, c])
    return ",".join(f"{a}-{b}" if a != b else str(a) for a, b in runs)


def gpu_local_cpus():
    """Per visible GPU (HIP's order), the CPUs local to it, from sysfs only
    (no HIP call): KFD topology nodes with SIMDs in node order -> the PCI
    device of each (domain, location_id = bus << 8 | dev << 3 | fn) ->
    /sys/bus/pci/devices/<bdf>/local_cpulist.  Cut by *_VISIBLE_DEVICES
    when that is a list of indices.  None if sysfs is unreadable."""
    import glob
    try:
        nodes = []
        for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(p) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            if int(props.get("simd_count", "0")) > 0:
                nodes.append((int(p.split("/")[-2]), int(props.get("domain", "0")), int(props["location_id"])))
        nodes.sort()
        cpus = []
        for _, dom, loc in nodes:
            bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7}"
            with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
                cpus.append(_parse_cpulist(f.read()))
    except (OSError, ValueError, KeyError):
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            try:
                cpus = [cpus[int(x)] for x in v.split(",") if x.strip() != ""]
            except (ValueError, IndexError):
                return None
    return cpus


def rank_cpu_sets(nranks, allowed, local=None, share_device=False):
    """Disjoint CPU sets for local ranks 0..nranks-1 (rank r drives GPU r,
    or GPU 0 for every rank with --share-device): each GPU's local CPUs
    within ``allowed`` (this process's affinity), split evenly between the
    ranks on the same set of local CPUs.  Falls back to an even split of
    ``allowed`` when the topology is unknown or the per-GPU sets overlap
    without being equal.  Returns (sets, source) or (None, reason) when
    there are fewer CPUs than ranks."""
    allowed = set(allowed)
    groups, source = None, "even-split"
    if local is not None and (share_device or len(local) >= nranks):
        per = [set(local[0 if share_device else r]) & allowed for r in range(nranks)]
        keys = {frozenset(s) for s in per}
        if all(per) and all(a == b or not (a & b) for a in keys for b in keys):
            groups, source = {}, "gpu-local"
            for r, s in enumerate(per):
                groups.setdefault(frozenset(s), []).append(r)
    if groups is None:
        groups = {frozenset(allowed): list(range(nranks))}
    out = [None] * nranks
    for cpus, ranks in groups.items():
        cl = sorted(cpus)
        k = len(ranks)
        if len(cl) < k:
            return None, f"{len(cl)} cpus for {k} ranks"
        for i, r in enumerate(ranks):
            out[r] = set(cl[i * len(cl) // k:(i + 1) * len(cl) // k])
    return out, source


def pin_rank(args):
    """Before the rank's first GPU call: pin this process to its disjoint
    share of the CPUs near its GPU (rank_cpu_sets; one host thread submits
    the rank's graph replays).  Only with more than one rank;
    PVNET_NO_PIN=1 turns it off.  Returns (cpulist string, source)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    cur = os.sched_getaffinity(0)
    if ws <= 1 or os.environ.get("PVNET_NO_PIN") == "1":
        return _fmt_cpulist(cur), "unpinned"
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    sets, source = rank_cpu_sets(lw, cur, None if args.dry_run else gpu_local_cpus(),
                                 share_device=args.share_device)
    if sets is None:
        return _fmt_cpulist(cur), f"unpinned ({source})"
    os.sched_setaffinity(0, sets[lr])
    return _fmt_cpulist(sets[lr]), source


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) outside torchrun: start the N ranks as child
    processes (the script again, RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1 and a free port) and wait for them.  This process
    makes no GPU call: it counts the devices from the KFD topology in sysfs
    and the *_VISIBLE_DEVICES masks (visible_gpus; torch.cuda.device_count()
    may fall back to hipGetDeviceCount, which initialises HIP before the
    fork) and fails if fewer than N are visible.  Rank 0
    prints the JSON line.  If a rank fails, the others (this process's own
    children, by PID) are terminated.  Returns the exit code."""
    import signal
    import socket
    import subprocess
    n = args.gpus
    if not args.dry_run and not args.share_device:
        have = visible_gpus()
        if have is not None and have < n:
            log(f"bench.py --gpus {n}: only {have} GPU(s) visible")
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n))
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    # rank 0's stdout is this process's (the JSON line); the others' goes to stderr
    procs = [subprocess.Popen(cmd, env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=None if r == 0 else sys.stderr) for r in range(n)]

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc, live = 0, list(procs)
    try:
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    log(f"rank {procs.index(p)} exited with {c}: stopping the other ranks")
                    stop()
            time.sleep(0.1)
    except KeyboardInterrupt:
        stop()
        raise
    return rc


def gather_rank_cpus(args, ws):
    """Every rank's CPU list (pin_rank), in rank order, for the line."""
    if ws <= 1:
        return [args.rank_cpus[0]]
    allc = [None] * ws
    dist.all_gather_object(allc, args.rank_cpus[0])
    return allc


def setup_dist(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"WORLD_SIZE {ws} != --gpus {args.gpus}")
    if args.dry_run:
        if ws > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
        return ws, rank, torch.device("cpu")
    if ws > 1 and args.share_device:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        return ws, rank, torch.device("cuda", 0)
    if ws > 1:
        if torch.cuda.device_count() <= local:
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but {torch.cuda.device_count()} GPU(s) visible")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return ws, rank, torch.device("cuda", local if ws > 1 else 0)


def field_seed(i, ws, nfields):
    """S(seed) of stream image i: the stream cycles through nfields * ws
    seeds, so rank i % ws holds exactly nfields of them."""
    return 1234 + i % (nfields * ws)


def make_fields(rank, ws, nfields, dev):
    """The rank's resident fields (network layout, f32), seed 1234 + rank + ws*f:
    views [1, ...] of one [nfields, ...] tensor each (so consecutive fields
    are also a batch: the stream_batched leg)."""
    from pvnet_amd import synth
    segs, vers, kps = [], [], []
    for f in range(nfields):
        fd = synth.synthetic_field(1234 + rank + ws * f)
        if f == 0:
            seg_all = torch.empty((nfields,) + fd["seg"].shape[1:], dtype=torch.float32, device=dev)
            ver_all = torch.empty((nfields,) + fd["vertex"].shape[1:], dtype=torch.float32, device=dev)
        seg_all[f].copy_(torch.from_numpy(fd["seg"][0]))
        ver_all[f].copy_(torch.from_numpy(fd["vertex"][0]))
        segs.append(seg_all[f:f + 1])
        vers.append(ver_all[f:f + 1])
        kps.append(fd["keypoints"])
    return segs, vers, np.stack(kps), int(fd["tn"])


def make_stream_fields(rank, ws, nfields, dev):
    """The rank's resident configs[3] frames: stream images rank + ws*f of
    pvnet_amd.synth.stream_field (full, occluded split, below min_num, above
    max_num, quadrant-occluded, empty, border-clipped, just above min_num)."""
    from pvnet_amd import synth
    segs, vers, kps, tns, kinds = [], [], [], [], []
    for f in range(nfields):
        fd = synth.stream_field(rank + ws * f)
        segs.append(torch.from_numpy(fd["seg"]).to(dev))
        vers.append(torch.from_numpy(fd["vertex"]).to(dev))
        kps.append(fd["keypoints"])
        tns.append(int(fd["tn"]))
        kinds.append(fd["kind"])
    return segs, vers, np.stack(kps), np.array(tns), kinds


def graph_stream(args, ws, rank, dev, steps, seed_base, vote, parts, per_step=None, lanes_state=None,
                 frames_per_call=1, stats=None):
    """The timed stream core: this rank's share (pvnet_amd.distributed.shard)
    of ws * steps * M images; one step = one hipGraph replay of M /
    frames_per_call calls of ``vote(j, seed, lane, outs)`` (the call at frame
    j writes rows j .. j + frames_per_call - 1 of each per-step output in
    ``outs``), --inflight of them at a time on their own streams; one gather
    of every image's result at the end of the timed region.  ``parts`` =
    [(shape, dtype)] of one image's result.  ``stats`` (a dict) receives the
    host seconds spent inside the timed graph.replay() calls.  Returns
    (elapsed s (max over ranks), local results [steps*M, ...] per part,
    gathered results per part (stream order), the capture stream)."""
    from pvnet_amd import distributed as D
    M, K = per_step or args.per_step, steps
    n_images = ws * K * M                          # the whole stream, sharded round-robin
    mine = D.shard(n_images, rank, ws)             # this rank's images, in stream order
    assert len(mine) == K * M and M % frames_per_call == 0
    NL = max(1, args.inflight)
    lanes = [new_stream(dev) for _ in range(NL)]
    outs = [torch.zeros((M,) + tuple(sh), dtype=dt, device=dev) for sh, dt in parts]
    local = [torch.zeros((K * M,) + tuple(sh), dtype=dt, device=dev) for sh, dt in parts]
    s = new_stream(dev)

    def step_body(seed0):
        for ln in lanes:
            ln.wait_stream(torch.cuda.current_stream())
        for c, j in enumerate(range(0, M, frames_per_call)):
            with torch.cuda.stream(lanes[c % NL]):
                vote(j, seed0 + 17 * j, c % NL, outs)
        for ln in lanes:
            torch.cuda.current_stream().wait_stream(ln)

    # warmup (eager: every lane's workspace sized, nothing is JIT-compiled)
    with torch.cuda.stream(s):
        for w in range(max(1, args.warmup)):
            step_body(seed_base + 1000 * w + rank * 7_919)
    torch.cuda.synchronize()
    graph = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            step_body(seed_base + 3 + rank * 1_000_003)
    graph.replay()                                 # one untimed replay (graph upload)
    torch.cuda.synchronize()

    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for k in range(K):
            h0 = time.perf_counter()
            graph.replay()
            host += time.perf_counter() - h0
            for loc, o in zip(local, outs):
                loc[k * M:(k + 1) * M].copy_(o)
        # the stream's one exchange: every image's result to every rank, in
        # stream order (pvnet_amd.distributed: RCCL all_gather over xGMI)
        if len(parts) == 1:
            allr = (D.gather_results(local[0], n_images, rank, ws),)
        else:
            allr = D.gather_results_multi(local, n_images, rank, ws)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mine_t = torch.tensor(mine, device=dev)
        for a_, l_ in zip(allr, local):
            assert torch.equal(a_[mine_t], l_), "gathered stream order differs from the shard"
    if stats is not None:
        stats["host_replay_s"] = host
    return elapsed, local, allr, s


def run_stream(args, ws, rank, dev, segs, vers, steps, seed_base, frames_per_call=1, stats=None):
    """The v3 stream: ransac_voting_layer_v3 on seg_pred/vertex_pred of
    resident field j % len(segs) per slot, its own workspace per lane.  With
    frames_per_call f > 1 one call votes f consecutive resident fields as a
    batch (segs / vers must then be consecutive views of one tensor).
    Returns (elapsed s (max over ranks), local keypoints [steps*M, 9, 2],
    lanes' workspaces, the capture stream, gathered keypoints)."""
    from pvnet_amd import ransac_voting_gpu as rvg
    NF = len(segs)
    f = frames_per_call
    works = [rvg.VotingWorkspace() for _ in range(max(1, args.inflight))]
    if f > 1:
        assert NF % f == 0
        seg_all = segs[0].as_strided((NF,) + tuple(segs[0].shape[1:]), segs[0].stride())
        ver_all = vers[0].as_strided((NF,) + tuple(vers[0].shape[1:]), vers[0].stride())
        assert all(segs[i].data_ptr() == seg_all[i].data_ptr() and vers[i].data_ptr() == ver_all[i].data_ptr()
                   for i in range(NF)), "batched frames must be consecutive views of one tensor"

    def vote(j, seed, lane, outs):
        if f == 1:
            rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], args.hn, _seed=seed,
                                                   _workspace=works[lane], out=outs[0][j:j + 1])
        else:
            i = j % NF
            rvg.ransac_voting_layer_v3_from_network(seg_all[i:i + f], ver_all[i:i + f], args.hn, _seed=seed,
                                                   _workspace=works[lane], out=outs[0][j:j + f])
    elapsed, local, allr, s = graph_stream(args, ws, rank, dev, steps, seed_base, vote,
                                           [((VN, 2), torch.float32)], frames_per_call=f, stats=stats)
    return elapsed, local[0], works, s, allr[0]


def stream_order_error(allkp, ws, nfields):
    """Max |keypoint - generating keypoint| over the gathered stream: image i
    (voted by rank i % ws) against S(field_seed(i)), so a result gathered into
    the wrong slot shows as an error of tens of pixels."""
    from pvnet_amd import synth
    seeds = [field_seed(i, ws, nfields) for i in range(nfields * ws)]
    ref = np.stack([synth.field_keypoints(sd) for sd in seeds]).astype(np.float32)
    got = allkp.cpu().numpy()
    return float(np.abs(got - ref[np.arange(got.shape[0]) % (nfields * ws)]).max())


def dry_run(args, ws, rank):
    """--dry-run (CPU, gloo): the launcher, the shard, the timed region's
    barriers, the gather, the max over ranks and the stream-order check, with
    each image's result = its field's generating keypoints (nothing is voted);
    rank 0 prints a line of the real run's form marked dry_run."""
    from pvnet_amd import distributed as D
    from pvnet_amd import synth
    K, M, NF = args.steps, args.per_step, max(1, args.fields)
    n_images = ws * K * M
    mine = D.shard(n_images, rank, ws)
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    local = torch.from_numpy(np.stack([synth.field_keypoints(field_seed(i, ws, NF)) for i in mine]).astype(np.float32))
    allkp = D.gather_results(local, n_images, rank, ws)
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    err = stream_order_error(allkp, ws, NF)
    if rank == 0:
        line = {"metric": "images/sec (480x640, 9 kp) vote->keypoint", "value": round(n_images / elapsed, 2),
                "unit": "images/sec", "n_gpus": ws, "steps": K, "warmup": args.warmup,
                "ms_per_step": round(elapsed / K * 1e3, 5), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "f32", "data": "none (dry run)", "dry_run": True,
                "config": {"workload": "dry run: launcher + shard + gather only, no voting", "global_batch": M * ws,
                           "per_gpu_batch_per_step": M, "stream_images": n_images},
                "stream_order_max_err_px": err, "stream_order_ok": err == 0.0,
                "rank_cpus": args.rank_cpus_all, "rank_cpus_source": args.rank_cpus[1]}
        assert line["n_gpus"] == args.gpus
        if not args.skip_cpu:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    faulthandler.enable()          # a host crash names its Python frame (DESIGN.md "Concurrent callers")
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args))
    args.rank_cpus = pin_rank(args)      # before any GPU call
    ws, rank, dev = setup_dist(args)
    args.rank_cpus_all = gather_rank_cpus(args, ws)
    if args.dry_run:
        return dry_run(args, ws, rank)
    from pvnet_amd import ransac_voting_gpu as rvg

    M, K, NF = args.per_step, args.steps, max(1, args.fields)
    n_images = ws * K * M
    segs, vers, kps, tn = make_fields(rank, ws, NF, dev)
    # local image j (stream image rank + ws * j) votes field j % NF: field_seed == 1234 + rank + ws * (j % NF)
    assert all(field_seed(rank + ws * j, ws, NF) == 1234 + rank + ws * (j % NF) for j in range(4 * NF))
    hs = {}
    elapsed, local, works, s, allkp = run_stream(args, ws, rank, dev, segs, vers, K, 0, stats=hs)
    # every gathered image against its field's generating keypoints: a result
    # in the wrong stream slot would be tens of pixels off
    order_err = stream_order_error(allkp, ws, NF)
    del allkp
    out_step = torch.zeros((M, VN, 2), dtype=torch.float32, device=dev)

    # sanity on the timed outputs: every local image against its field's
    # generating keypoints (the noisy field limits LS accuracy to ~1-2 px;
    # parity is in tests/)
    lk = local.cpu().numpy()
    err = float(np.abs(lk - kps[np.arange(K * M) % NF]).max())
    if ws > 1:
        e = torch.tensor([err], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        err = float(e.item())
    if err > 5.0:
        raise SystemExit(f"keypoint error {err} px > 5 on the synthetic fields (tn={tn})")

    # the same stream with 4 consecutive resident frames per call (one batched
    # v3 call: its 4 kernel nodes per 4 frames instead of per frame): separates
    # the host's per-node graph submission from the GPU's work per frame
    sb = None
    if not args.skip_batched:
        sb = stream_batched(args, ws, rank, dev, segs, vers, kps, 4)

    # configs[3]: the Occlusion-LINEMOD-like stream (mixed masks), the same
    # sharding and gather, fewer steps
    c3 = c4 = None
    if not args.skip_config3:
        c3 = stream_config3(args, ws, rank, dev)
        c4 = stream_config4(args, ws, rank, dev)

    # dominant kernels' durations with hipEvents on the streams they run on
    seeds = [rank * 1_000_003 + 17 * k + 3 for k in range(min(K * 5, 100))]
    vote_ms, compact_ms = time_vote_kernel(rvg, segs, vers, args.hn, seeds, works[0], out_step, s)
    # per-image latency: 32 images one after another on one stream (rotating fields)
    NLAT = 32
    lat = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(lat, stream=s):
            for j in range(NLAT):
                rvg.ransac_voting_layer_v3_from_network(segs[j % NF], vers[j % NF], args.hn, _seed=seeds[j % len(seeds)],
                                                       _workspace=works[0], out=out_step[j % M:j % M + 1])
    lat.replay()
    torch.cuda.synchronize()
    lat_runs = []                      # the median of 5 timed replays (one replay alone varies by ~1 us/image)
    for _ in range(5):
        t1 = time.perf_counter()
        lat.replay()
        torch.cuda.synchronize()
        lat_runs.append((time.perf_counter() - t1) / NLAT * 1e3)
    latency_ms = float(np.median(lat_runs))
    res = dict(elapsed=elapsed, vote_ms=vote_ms, compact_ms=compact_ms, tn=tn, latency_ms=latency_ms,
               n_images=n_images, config3=c3, config4=c4, order_err=order_err, batched=sb,
               host_ms_per_replay=hs["host_replay_s"] / K * 1e3)
    if rank == 0:
        report(args, ws, res, err, dev)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


def kernel_nodes(frames_per_call=1, hn=512):
    """Kernel launches (graph nodes) of one v3 call on frames_per_call
    480x640 frames, as the library reports them (pv_v3_kernel_launches)."""
    from pvnet_amd import _lib
    return int(_lib.load().pv_v3_kernel_launches(frames_per_call, H, W, VN, hn))


def stream_batched(args, ws, rank, dev, segs, vers, kps, f):
    """stream_batched<f>: the headline stream's frames, sharding, lanes and
    gather, but each lane call votes f consecutive resident frames as one
    batch (RV:531's per-image loop is batched in the reference's pipeline
    too): one call's kernel nodes per f frames.  Not the headline (batch-1 frames)."""
    K, M, NF = args.steps, args.per_step, len(segs)
    hs = {}
    elapsed, local, _, _, _ = run_stream(args, ws, rank, dev, segs, vers, K, 77_000, frames_per_call=f, stats=hs)
    n = ws * K * M
    err = float(np.abs(local.cpu().numpy() - kps[np.arange(K * M) % NF]).max())
    return dict(images_per_s=round(n / elapsed, 1), ms_per_step=round(elapsed / K * 1e3, 4), steps=K,
                frames_per_call=f, per_gpu_batch_per_step=M, kernel_nodes_per_frame=kernel_nodes(f) / f,
                host_ms_per_replay=round(hs["host_replay_s"] / K * 1e3, 4), max_kp_err_px=round(err, 4),
                note="the headline stream (same fields, 8 lanes, one graph replay per %d frames) with %d consecutive "
                     "frames per ransac_voting_layer_v3 call; host_ms_per_replay = host time inside "
                     "graph.replay() (the runtime's submission of the replay's kernel nodes)" % (M, f))


def stream_config3(args, ws, rank, dev, steps=8):
    """configs[3] (BASELINE.json): the stream of mixed Occlusion-LINEMOD-like
    frames (synth.stream_field, 8 kinds cycling) sharded round-robin over the
    ranks, voted through the same graph-replayed lanes, keypoints gathered
    once; images/s over all ranks (max-over-ranks wall time)."""
    NF = max(8, args.fields)
    segs, vers, kps, tns, kinds = make_stream_fields(rank, ws, NF, dev)
    elapsed, local, _, _, _ = run_stream(args, ws, rank, dev, segs, vers, steps, 50_000)
    n = ws * steps * args.per_step
    lk = local.cpu().numpy()
    j = np.arange(lk.shape[0]) % NF
    voted = tns[j] >= 100
    zeros_ok = bool(np.all(lk[~voted] == 0))
    # distance to the generating keypoints per mask kind (a sanity figure:
    # the field's 0.05 rad noise and 20 % outliers limit least squares far
    # from small or clipped masks; parity is tests/test_gpu_stream.py)
    e = np.linalg.norm(lk - kps[j], axis=-1).max(-1)
    err = {k: round(float(np.median(e[[kinds[x] == k for x in j] & voted])), 3)
           for k in dict.fromkeys(kinds) if np.any([kinds[x] == k for x in j] & voted)}
    del segs, vers
    torch.cuda.empty_cache()
    return dict(images_per_s=round(n / elapsed, 1), ms_per_step=round(elapsed / steps * 1e3, 4), steps=steps,
                per_gpu_batch_per_step=args.per_step, n_gpus=ws, stream_images=n,
                kinds={k: int(sum(1 for x in kinds if x == k)) for k in dict.fromkeys(kinds)},
                tn_range=[int(tns.min()), int(tns.max())], zeros_path_ok=zeros_ok,
                median_kp_err_px_by_kind=err,
                note="configs[3] workload: full / occluded split / below min_num (zeros path, RV:537-540) / above "
                     "max_num (Bernoulli downsampling, RV:543-546) / quadrant-occluded / empty / border-clipped / "
                     "just above min_num frames cycling, images sharded round-robin over ranks, one all_gather of "
                     "keypoints; parity: tests/test_gpu_stream.py")


YCB_K = np.array([[1066.778, 0.0, 312.9869], [0.0, 1067.487, 241.3109], [0.0, 0.0, 1.0]])   # the YCB-Video camera


def make_ycb_fields(rank, ws, nfields, dev, kp=21):
    """The rank's resident configs[4] frames: 21 model points (a seeded
    12 cm object) at a random pose 0.9-1.1 m in front of the YCB camera,
    projected to 21 keypoints; S(seed)-style field around them (disk r 97.5,
    ~29.9k foreground pixels, 0.05 rad noise, 20 % outliers), network layout
    f32.  Returns (segs, vers, model points, poses [nf, 3, 4])."""
    from pvnet_amd import synth
    p3 = np.random.default_rng(5).uniform(-0.06, 0.06, size=(kp, 3))
    segs, vers, poses = [], [], []
    for f_ in range(nfields):
        rng = np.random.default_rng(90_000 + rank + ws * f_)
        a = rng.normal(size=3) * 0.4
        th = np.linalg.norm(a)
        kx = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]) / th
        R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
        t = np.array([rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05), rng.uniform(0.9, 1.1)])
        X = p3 @ R.T + t
        k2 = np.stack([YCB_K[0, 0] * X[:, 0] / X[:, 2] + YCB_K[0, 2], YCB_K[1, 1] * X[:, 1] / X[:, 2] + YCB_K[1, 2]], 1)
        fd = synth.synthetic_field(90_000 + rank + ws * f_, vn=kp, keypoints=k2,
                                   center=(float(k2[:, 0].mean()), float(k2[:, 1].mean())))
        segs.append(torch.from_numpy(fd["seg"]).to(dev))
        vers.append(torch.from_numpy(fd["vertex"]).to(dev))
        poses.append(np.concatenate([R, t[:, None]], 1))
    return segs, vers, p3, np.stack(poses)


def stream_config4(args, ws, rank, dev, steps=4, per_step=32, nfields=16):
    """configs[4] (BASELINE.json): the YCB-Video stream sharded round-robin
    over the ranks; per image ransac_voting_layer_v3 (hn 512) from the
    network layout, estimate_voting_distribution_with_mean (16 x 256
    hypotheses) on argmax(seg) and the strided vertex view, and the
    uncertainty PnP of the 21 keypoints; one gather of (keypoints [21, 2],
    covariances [21, 2, 2], pose [3, 4]) per image in stream order.  Same
    graph-replayed lanes as the headline stream; images/s over all ranks."""
    from pvnet_amd import extend_utils as eu
    from pvnet_amd import ransac_voting_gpu as rvg
    KP = 21
    segs, vers, p3, poses = make_ycb_fields(rank, ws, nfields, dev, KP)
    tp3 = torch.from_numpy(p3).to(dev)
    tK = torch.from_numpy(YCB_K).to(dev)
    NL = max(1, args.inflight)
    w1 = [rvg.VotingWorkspace() for _ in range(NL)]
    w2 = [rvg.VotingWorkspace() for _ in range(NL)]

    def vote(j, seed, lane, outs):
        seg, ver = segs[j % nfields], vers[j % nfields]
        b, c, h, w = ver.shape
        kp = rvg.ransac_voting_layer_v3_from_network(seg, ver, args.hn, _seed=seed, _workspace=w1[lane],
                                                     out=outs[0][j:j + 1])
        mask = seg.argmax(1)
        vertex = ver.permute(0, 2, 3, 1).view(b, h, w, KP, 2)
        mean, cov = rvg.estimate_voting_distribution_with_mean(mask, vertex, kp, _workspace=w2[lane], _seed=seed + 1)
        outs[1][j:j + 1].copy_(cov)
        outs[2][j:j + 1].copy_(eu.pose_from_voting(mean, cov, tp3, tK))
    parts = [((KP, 2), torch.float32), ((KP, 2, 2), torch.float32), ((3, 4), torch.float64)]
    elapsed, local, allr, _ = graph_stream(args, ws, rank, dev, steps, 70_000, vote, parts, per_step=per_step)
    n = ws * steps * per_step
    Rt = local[2].cpu().numpy()
    j = np.arange(Rt.shape[0]) % nfields
    terr = np.abs(Rt[:, :, 3] - poses[j][:, :, 3]).max(1)
    del segs, vers
    torch.cuda.empty_cache()
    return dict(images_per_s=round(n / elapsed, 1), ms_per_step=round(elapsed / steps * 1e3, 4), steps=steps,
                per_gpu_batch_per_step=per_step, n_gpus=ws, stream_images=n, keypoints=KP,
                gathered=[list(a.shape) for a in allr],
                covariances_finite=bool(torch.isfinite(local[1]).all()),
                max_translation_err_m=round(float(terr.max()), 5), median_translation_err_m=round(float(np.median(terr)), 5),
                stages="v3 (hn 512) + EVD with mean (16 x 256) + uncertainty PnP (21 points) per image, graph-replayed "
                       "lanes; (keypoints, covariances, pose) gathered in stream order",
                note="configs[4] workload: YCB-Video-like 480x640 frames (21 keypoints of a 12 cm object 0.9-1.1 m "
                     "from the YCB camera, ~29.9k foreground px), images sharded round-robin over ranks; error vs "
                     "the generating pose; parity: tests/test_gpu_stream.py::test_config4_stream_*")


def time_vote_kernel(rvg, segs, vers, hn, seeds, work, out, stream):
    """Per-launch durations of the vote kernel (k_vote_mfma) and of the
    compaction (k_fg_count + k_compact): hipEvents the library records right
    before / after them on the stream they are launched on (the compaction is
    a call's first work: its start is an event recorded just before the
    call), over eager calls cycling through the resident fields (events
    inside a captured graph do not time the nodes between them).
    Returns (vote ms [n], compaction ms [n])."""
    from pvnet_amd import _lib
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in seeds]
    with torch.cuda.stream(stream):
        for e4 in ev:           # materialise the hipEvent_t handles
            for e in e4:
                e.record(stream)
        torch.cuda.synchronize()
        for k, (a, b, c0, c1) in enumerate(ev):
            c0.record(stream)
            dd = _lib.V3Diag(ev_vote_begin=a.cuda_event, ev_vote_end=b.cuda_event, ev_compact_end=c1.cuda_event)
            _raw_v3(rvg, segs[k % len(segs)], vers[k % len(vers)], hn, seeds[k], work, out[k % out.shape[0]], dd)
    torch.cuda.synchronize()
    return (np.array([a.elapsed_time(b) for a, b, _, _ in ev]), np.array([c0.elapsed_time(c1) for _, _, c0, c1 in ev]))


def _raw_v3(rvg, seg, ver, hn, seed, work, out, dd):
    """ransac_voting_layer_v3_from_network with per-kernel timing events."""
    import ctypes
    from pvnet_amd import _lib
    b, c, h, w = ver.shape
    vertex = ver.permute(0, 2, 3, 1).view(b, h, w, c // 2, 2)
    d = rvg._desc(seg, vertex, seg=True)
    prm = rvg._params(hn, 0.99, 0.99, 100, 100, 30000, seed)
    L = _lib.load()
    nbytes = L.pv_v3_workspace_size(b, h, w, c // 2, hn)
    wsb = work.get(ver.device, nbytes)
    try:
        code = L.pv_ransac_voting_v3(ctypes.byref(d), ctypes.byref(prm), out.data_ptr(), wsb.data_ptr(), nbytes,
                                     ctypes.byref(dd), torch.cuda.current_stream(ver.device).cuda_stream)
    finally:
        work.done(ver.device)
    _lib.check(code, "pv_ransac_voting_v3")
    return out


def measure_u1(dev, hn=512, reps=100):
    """API-faithful voting_for_hypothesis (dense u8 [hn,vn,tn] write) on one
    S(1234) image: the kernel the north star's HBM roofline names (U1).
    Timed on the launching stream with hipEvents around U1_TIMED replays of a
    hipGraph of `reps` calls, queued behind U1_WARM untimed ones: the device
    time per call in the sustained steady state, where each launch's 137.6 MB drain to HBM behind the next
    one (a launch alone on an idle device partly lands in the 256 MiB
    Infinity Cache and measures faster); rocprof's kernel trace of the same
    command times these launches (the only other ones are the 5 warm-up calls)."""
    from pvnet_amd import ransac_voting as rv
    from pvnet_amd import synth
    f = synth.synthetic_field(1234)
    m = np.argmax(f["seg"][0], 0) == 1
    rows, cols = np.nonzero(m)
    coords = torch.from_numpy(np.stack([cols, rows], 1).astype(np.float32)).to(dev)
    direct = torch.from_numpy(np.ascontiguousarray(
        f["vertex"][0].reshape(VN, 2, H, W)[:, :, rows, cols].transpose(2, 0, 1))).to(dev)
    tn = coords.shape[0]
    idxs = torch.randint(0, tn, (hn, VN, 2), dtype=torch.int32, device=dev)
    hyp = rv.generate_hypothesis(direct, coords, idxs)
    inl = torch.empty((hn, VN, tn), dtype=torch.uint8, device=dev)
    s = new_stream(dev)
    with torch.cuda.stream(s):
        for _ in range(5):
            rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
    torch.cuda.synchronize()
    # `reps` launches back to back in one hipGraph (no host gaps between
    # them: the device time per launch that rocprof's kernel trace measures)
    g = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                rv.voting_for_hypothesis_dense(direct, coords, hyp, inl, 0.99)
    g.replay()
    torch.cuda.synchronize()
    # sustained: U1_WARM replays back to back untimed (the clocks and the
    # Infinity Cache reach their steady state: the first replays after an
    # idle device run 36 -> 31 us per launch, tools/u1_replays.py), then
    # U1_TIMED replays timed -- queued behind the warm ones, so the events
    # see kernel after kernel, the period rocprof's trace shows
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        for _ in range(U1_WARM):
            g.replay()
        a.record(s)
        for _ in range(U1_TIMED):
            g.replay()
        b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / (reps * U1_TIMED)
    nbytes = 8 * tn * VN + 8 * tn + 8 * hn * VN + hn * VN * tn      # SURVEY 8(d) U1 algorithmic bytes
    return dict(kernel="k_vote_bytes<DENSE> (pv_voting_for_hypothesis)", bytes_per_launch=nbytes,
                traffic=pmc_traffic("k_vote_bytes"), ms=ms,
                achieved_gbs=nbytes / (ms * 1e-3) / 1e9, peak_gbs=HBM_PEAK_GBS,
                frac=nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, hn=hn, tn=tn)


def measure_u4(dev, reps=20):
    """U4: estimate_voting_distribution_with_mean (RV:333-406)
    on S(1234) -- 16 rounds x 256 hypotheses = one vote/count launch over 4096
    hypotheses per keypoint, then the covariance reduction (k_evd_with_mean).
    hipEvents the library records on the launching stream around the vote
    kernel (pv_estimate_voting_distribution_with_mean_diag), plus one after
    the call for the reduction; eager calls, medians over `reps`."""
    import ctypes
    from pvnet_amd import _lib
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd import synth
    f = synth.synthetic_field(1234)
    mask = torch.from_numpy(np.argmax(f["seg"], 1)).to(dev)
    vertex = torch.from_numpy(np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, H, W, VN, 2))).to(dev)
    mean = torch.from_numpy(f["keypoints"].astype(np.float32)[None]).to(dev)
    work = rvg.VotingWorkspace()
    L = _lib.load()
    s = new_stream(dev)
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(5)) for _ in range(reps + 3)]
    cov = torch.empty((1, VN, 2, 2), dtype=torch.float32, device=dev)
    with torch.cuda.stream(s):
        for e5 in ev:
            for e in e5:
                e.record(s)
        torch.cuda.synchronize()
        for k, (c0, c1, v0, v1, e1) in enumerate(ev):
            d, prm, nbytes, keep, _ = rvg._evd_common(mask, vertex, 256, 4096, 0.99, 20, 30000, 128, None, None,
                                                       1000 + k, work)
            dd = _lib.V3Diag(ev_vote_begin=v0.cuda_event, ev_vote_end=v1.cuda_event, ev_compact_end=c1.cuda_event)
            ws = work.get(dev, nbytes)
            c0.record(s)
            try:
                _lib.check(L.pv_estimate_voting_distribution_with_mean_diag(
                    ctypes.byref(d), ctypes.byref(prm), mean.data_ptr(), cov.data_ptr(), ws.data_ptr(), nbytes,
                    ctypes.byref(dd), s.cuda_stream), "pv_estimate_voting_distribution_with_mean_diag")
            finally:
                work.done(dev)
            e1.record(s)
    torch.cuda.synchronize()
    ev = ev[3:]                                   # the first calls size the workspace and warm up
    vote = np.array([v0.elapsed_time(v1) for _, _, v0, v1, _ in ev])
    red = np.array([v1.elapsed_time(e1) for _, _, _, v1, e1 in ev])
    call = np.array([c0.elapsed_time(e1) for c0, _, _, _, e1 in ev])
    tn = int(f["tn"])
    flops = 12.0 * 4096 * VN * tn                # 16 x U2 at hn 256: 12 FLOP per (hypothesis, keypoint, pixel)
    vm = float(np.median(vote))
    achieved = flops / (vm * 1e-3) / 1e12
    c = cov.cpu().numpy()
    return dict(bound="valu", kernel="k_vote_mfma at n_hyp 4096 (U4's 16 x 256 hypotheses) + k_evd_with_mean",
                achieved=round(achieved, 2), peak=FP32_VECTOR_PEAK_TFLOPS, unit="TFLOP/s",
                frac=round(achieved / FP32_VECTOR_PEAK_TFLOPS, 4), avg_kernel_ms=round(vm, 5),
                flop_per_launch=flops, reduce_ms=round(float(np.median(red)), 5),
                call_ms=round(float(np.median(call)), 5), tn=tn, hyp=4096, samples=len(ev),
                traffic=pmc_traffic("k_vote_mfma_evd"), cov_finite=bool(np.isfinite(c).all()),
                note="estimate_voting_distribution_with_mean on S(1234) (tn 29,861, 9 kp): FLOP = 16 x 12 x 256 x vn "
                     "x tn (SURVEY 8(d) U4) / the median vote-kernel time between hipEvents the library records "
                     "around it on its stream (eager calls); reduce_ms = the covariance reduction "
                     "(k_evd_with_mean) to the call's end, call_ms = the whole call (compaction + hypotheses + "
                     "vote + reduction); rocprof durations of the same command: %s" % STATS_FILE)


def config2_fields(b=32):
    """configs[2]-shaped batch: 32 fields whose foreground spans ~2k..30k
    pixels (13 disk radii, cycling: 'all 13 objects')."""
    from pvnet_amd import synth
    return [synth.synthetic_field(5000 + i, radius=25.0 + 72.5 * (i % 13) / 12.0) for i in range(b)]


def measure_batch(dev, b=32, hn=512, steps=10):
    """configs[2]'s voting half on its own: one call votes the batch of 32
    mixed-size fields (fp32 network layout), hipGraph of `steps` calls."""
    from pvnet_amd import ransac_voting_gpu as rvg
    fs = config2_fields(b)
    seg = torch.from_numpy(np.concatenate([f["seg"] for f in fs])).to(dev)
    ver = torch.from_numpy(np.concatenate([f["vertex"] for f in fs])).to(dev)
    work = rvg.VotingWorkspace()
    out = torch.zeros((steps, b, VN, 2), dtype=torch.float32, device=dev)
    s = new_stream(dev)
    with torch.cuda.stream(s):
        for k in range(3):
            rvg.ransac_voting_layer_v3_from_network(seg, ver, hn, _seed=k, _workspace=work, out=out[0])
    torch.cuda.synchronize()
    g = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for k in range(steps):
                rvg.ransac_voting_layer_v3_from_network(seg, ver, hn, _seed=100 + k, _workspace=work, out=out[k])
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    err = float(np.abs(out.cpu().numpy() - np.stack([f["keypoints"] for f in fs])[None]).max())
    return dict(images_per_s=round(b * steps / dt, 1), ms_per_batch=round(dt / steps * 1e3, 4), batch=b,
                tn_range=[min(f["tn"] for f in fs), max(f["tn"] for f in fs)], max_kp_err_px=round(err, 4),
                note="voting only; error vs the generator's keypoints (the smallest disks, tn~2k, alone limit it "
                     "to ~29 px; parity: tests/test_gpu_parity.py::test_v3_config2_batch32_mixed)")


def measure_pnp(dev, b=1024, reps=10, cpu_images=8):
    """configs[4]'s last stage: uncertainty PnP (pv_uncertainty_pnp, one wave
    per image, fp64) on b synthetic LINEMOD-camera images of 9 box keypoints
    with anisotropic covariances; timed with hipEvents over `reps` launches.
    Beside it the CPU oracle (oracle/pnp.py: the same P3P + Ceres-LM
    restatement in numpy) on a small sample, images/s."""
    from pvnet_amd import extend_utils as eu
    rng = np.random.default_rng(0)
    K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])
    p3 = np.concatenate([np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)]) * 0.05,
                         np.zeros((1, 3))])
    p2 = np.empty((b, 9, 2), np.float32)
    cov = np.empty((b, 9, 2, 2), np.float32)
    for i in range(b):
        a = rng.normal(size=3)
        th = np.linalg.norm(a)
        k = a / th
        kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
        X = p3 @ R.T + np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.6, 1.0)])
        m = rng.normal(size=(9, 2, 2))
        cov[i] = m @ m.transpose(0, 2, 1) + 0.05 * np.eye(2)
        p2[i] = np.stack([K[0, 0] * X[:, 0] / X[:, 2] + K[0, 2], K[1, 1] * X[:, 1] / X[:, 2] + K[1, 2]], 1) \
            + rng.normal(size=(9, 2)) * 0.5
    tp2, tcov = torch.from_numpy(p2).to(dev), torch.from_numpy(cov).to(dev)
    tp3, tK = torch.from_numpy(p3).to(dev), torch.from_numpy(K).to(dev)
    eu.uncertainty_pnp_batch(tp2, tcov, tp3, tK)
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        eu.uncertainty_pnp_batch(tp2, tcov, tp3, tK)
    e.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(e) / reps
    from oracle import pnp as P
    t0 = time.perf_counter()
    for i in range(cpu_images):
        P.uncertainty_pnp(p2[i], P.weights_from_cov(cov[i]), p3, K)
    cpu = cpu_images / (time.perf_counter() - t0)
    return dict(images_per_s=round(b / (ms * 1e-3), 1), ms_per_batch=round(ms, 4), batch=b, keypoints=9,
                cpu_oracle_images_per_s=round(cpu, 2), cpu_sample=f"{cpu_images} images, 1 thread, numpy")


def measure_pose(dev, b=32, steps=5):
    """configs[4]'s path on the device, keypoints -> covariances -> poses:
    ransac_voting_layer_v3 + estimate_voting_distribution_with_mean (16
    rounds x 256 hypotheses) + uncertainty PnP, for a batch of b synthetic
    fields whose 9 keypoints are a 10 cm box projected by the LINEMOD camera
    at random poses; captured as one hipGraph, `steps` replays timed."""
    from pvnet_amd import extend_utils as eu
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd import synth
    rng = np.random.default_rng(3)
    K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])
    # 8 box corners + an off-centre ninth point (a centred one is collinear
    # with opposite corners: P3P has no solution on such triples)
    p3 = np.concatenate([np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)]) * 0.05,
                         np.array([[0.012, -0.017, 0.009]])])
    fs, ts = [], []
    for i in range(b):
        a = rng.normal(size=3) * 0.4
        th = np.linalg.norm(a)
        k = a / th
        kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
        t = np.array([rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05), rng.uniform(0.7, 0.9)])
        X = p3 @ R.T + t
        kp = np.stack([K[0, 0] * X[:, 0] / X[:, 2] + K[0, 2], K[1, 1] * X[:, 1] / X[:, 2] + K[1, 2]], 1)
        c = kp[8]
        fs.append(synth.synthetic_field(700 + i, keypoints=kp, center=(float(c[0]), float(c[1]))))
        ts.append(t)
    seg = torch.from_numpy(np.concatenate([f["seg"] for f in fs])).to(dev)
    ver = torch.from_numpy(np.concatenate([f["vertex"] for f in fs])).to(dev)
    bb, c2, h, w = ver.shape
    vertex = ver.permute(0, 2, 3, 1).view(bb, h, w, c2 // 2, 2)
    mask = seg.argmax(1)
    tp3, tK = torch.from_numpy(p3).to(dev), torch.from_numpy(K).to(dev)
    w1, w2 = rvg.VotingWorkspace(), rvg.VotingWorkspace()

    def once():
        mean = rvg.ransac_voting_layer_v3(mask, vertex, 512, _workspace=w1, _seed=11)
        mean, cov = rvg.estimate_voting_distribution_with_mean(mask, vertex, mean, _workspace=w2, _seed=12)
        return eu.uncertainty_pnp_batch(mean, cov, tp3, tK, mode="cov", diag=pd)
    pd = {}
    s = new_stream(dev)
    with torch.cuda.stream(s):
        Rt = once()
    torch.cuda.synchronize()
    g = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            Rt = once()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    terr = np.abs(Rt.cpu().numpy()[:, :, 3] - np.array(ts)).max(1)
    return dict(images_per_s=round(b / dt, 1), ms_per_batch=round(dt * 1e3, 4), batch=b,
                max_translation_err_m=round(float(terr.max()), 5), median_translation_err_m=round(float(np.median(terr)), 5),
                p3p_ok=int(pd["p3p_ok"].sum()), pnp_status=np.bincount(pd["status"].cpu().numpy(), minlength=7).tolist(),
                stages="v3 (hn 512) + EVD with mean (16 x 256 hypotheses) + uncertainty PnP (P3P + LM), one hipGraph",
                note="synthetic box-keypoint fields (0.05 rad noise, 20% outliers); error vs the generating pose")


def measure_e2e_config4(dev, batch=32, iters=10):
    """configs[4] end to end on one GPU: the YCB-Video network PVnet(42, 2)
    (21 keypoints; MR:7-79 with ver_dim 42) in the fp16 channels-last
    inference form, then ransac_voting_layer_v3 from its outputs,
    estimate_voting_distribution_with_mean (16 rounds x 256 hypotheses) on
    argmax(seg) and the strided vertex view, and the uncertainty PnP of all
    21 keypoints -- one hipGraph per batch of 32 480x640 frames.
    Random-init weights (none ship with the reference): timing only."""
    from pvnet_amd import extend_utils as eu
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd.network import PVNet, PVNetInference
    torch.manual_seed(0)
    H, W, KP = 480, 640, 21
    net = PVNetInference(PVNet(2 * KP, 2).eval()).to(dev).half().to(memory_format=torch.channels_last)
    x = torch.randn(batch, 3, H, W, device=dev).half().contiguous(memory_format=torch.channels_last)
    rng = np.random.default_rng(5)
    p3 = torch.from_numpy(rng.uniform(-0.06, 0.06, size=(KP, 3))).to(dev)
    K = torch.tensor([[1066.778, 0.0, 312.9869], [0.0, 1067.487, 241.3109], [0.0, 0.0, 1.0]],
                     dtype=torch.float64, device=dev)              # the YCB-Video camera
    w1, w2 = rvg.VotingWorkspace(), rvg.VotingWorkspace()

    def once():
        with torch.no_grad():
            seg, ver = net(x)
            mean = rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _workspace=w1, _seed=13)
            mask = seg.argmax(1)
            vertex = ver.permute(0, 2, 3, 1).view(batch, H, W, KP, 2)
            mean, cov = rvg.estimate_voting_distribution_with_mean(mask, vertex, mean, _workspace=w2, _seed=14)
            return eu.uncertainty_pnp_batch(mean, cov, p3, K, mode="cov")

    s = new_stream(dev)
    with torch.cuda.stream(s):
        for _ in range(2):
            once()
    torch.cuda.synchronize()
    g = new_graph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            Rt = once()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    return dict(images_per_s=round(batch / dt, 1), ms_per_batch=round(dt * 1e3, 4), batch=batch, keypoints=KP,
                backbone="PVnet(42, 2) fp16 channels-last inference form", poses_finite=int(torch.isfinite(Rt).all(-1).all(-1).sum()),
                stages="backbone + v3 (hn 512) + EVD with mean (16 x 256) + uncertainty PnP (21 points), one hipGraph",
                note="random-init weights (none ship with the reference): timing only; parity of each stage: "
                     "tests/test_backbone.py (PVnet(42, 2) vs G4), tests/test_gpu_pnp.py, tests/test_gpu_parity.py")


FP16_MFMA_DENSE_TFLOPS = 2500.0      # MI355X dense fp16/bf16 matrix peak (no sparsity)
FP32_MATRIX_TFLOPS = 157.3           # f32 MFMA = the vector peak (MI355X_MICROARCH.md)
BACKBONE_GFLOP = 144.9               # ResNet-18 OS8 seg+vertex forward at 480x640


def measure_e2e(dev, half=False, batch=1, iters=30, hn=512, form=None):
    """configs[1] (fp32, batch 1) / configs[2] (fp16 backbone, batch 32):
    the ResNet-18 seg+vector-field forward (PyTorch-ROCm, MIOpen,
    channels_last) and the HIP v3 layer on the network's own outputs (fp16
    outputs are voted in fp32: the compaction widens them), captured together
    as one hipGraph.  The outputs are channels_last, so the [b,h,w,vn,2] view
    of vertex_pred is contiguous and no copy is made.  Random-init weights
    (the reference ships none): the foreground is whatever the seeded network
    predicts, so this times the path, not accuracy.  The backbone alone is
    timed too (its own graph) for its fraction of the matrix peak."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd.network import PVNet, PVNetInference, fold_batchnorm
    torch.backends.cudnn.benchmark = True      # MIOpen: search the convolution algorithms once
    torch.manual_seed(0)
    dt_ = torch.float16 if half else torch.float32
    # PVNetInference: BatchNorm folded into the convolutions and each decoder
    # upsampling fused with the cat after it in one HIP pass
    # (pv_upsample2x_cat_f16/_f32), parity-tested against G4.  Interleaved
    # A/B (tools/e2e_ab.py): fp16 batch 32 plain 1.82k, folded 2.13k,
    # inference 2.78k images/s; f32 batch 1 plain 488, folded 480, inference
    # 511 (folding alone does not pay in f32: the bias pass costs the BN pass).
    # Backbone alone, fp16 batch 32 (tools/backbone_ab.py, profiles/r03_backbone_ab.txt):
    # module epilogues 10.4 ms, fused epilogues 8.8 ms, + fused decoder tail 8.2 ms.
    form = form or "inference"
    net = PVNet(18, 2).eval()
    if form == "folded":
        net = fold_batchnorm(net)
    elif form == "inference":
        net = PVNetInference(net)
    net = net.to(dev).to(dtype=dt_, memory_format=torch.channels_last)
    x = torch.randn(batch, 3, H, W, device=dev).to(dtype=dt_, memory_format=torch.channels_last)
    ws = rvg.VotingWorkspace()
    out = torch.zeros((batch, VN, 2), dtype=torch.float32, device=dev)
    diag = {}

    def backbone():
        with torch.no_grad():
            return net(x)

    def once():
        sg, v = backbone()
        return rvg.ransac_voting_layer_v3_from_network(sg, v, hn, _workspace=ws, max_num=30000, _seed=7, out=out)

    def timed(fn):
        s = new_stream(dev)
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        g = new_graph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                fn()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters

    with torch.no_grad():
        sg, v = backbone()
        rvg.ransac_voting_layer_v3_from_network(sg, v, hn, _workspace=ws, _seed=7, _diag=diag)
    torch.cuda.synchronize()
    tn = diag["tn"].cpu().numpy()
    dt = timed(once)
    dtb = timed(backbone)
    peak = FP16_MFMA_DENSE_TFLOPS if half else FP32_MATRIX_TFLOPS
    bb_tf = BACKBONE_GFLOP * batch / dtb / 1e3
    return dict(images_per_s=round(batch / dt, 1), ms_per_batch=round(dt * 1e3, 4), batch=batch,
                backbone_dtype="float16" if half else "float32", voting_dtype="float32", backbone_form=form,
                backbone_ms_per_batch=round(dtb * 1e3, 4), backbone_gflop_per_image=BACKBONE_GFLOP,
                backbone_tflops=round(bb_tf, 1), backbone_matrix_peak_tflops=peak,
                backbone_frac_of_matrix_peak=round(bb_tf / peak, 4),
                voting_ms_per_batch=round((dt - dtb) * 1e3, 4), foreground_px=[int(tn.min()), int(tn.max())],
                note="random-init weights (none ship with the reference): timing only; images/s covers backbone + "
                     "v3 in one graph; backbone_form inference = pvnet_amd.network.PVNetInference (BN folded). fp16: "
                     "every convolution is a HIP matrix-core kernel with its epilogue fused (stem 7x7/2 as an s2d "
                     "4x4 conv, layer1 halo kernel, layer2-4 / fc / conv8s implicit GEMM with the downsample 1x1 "
                     "summed into conv2 and conv8s reading [xfc, x8s] from the two maps, the decoder's up2 + cat + "
                     "conv steps and convraw + 1x1 head; DESIGN.md 7a); f32: MIOpen convolutions + one HIP epilogue "
                     "pass each, HIP upsample+cat, convraw's LeakyReLU + 1x1 conv as one matrix-core pass; the "
                     "backbone alone is a separate graph")


def measure_kp_vs_ref(dev):
    """The metric's '2D kp L2 err vs ref': the device v3 with the golden
    fixtures' injected pixel pairs on the fixtures' own inputs (the LINEMOD
    'cat' demo field and S(1234)), against the keypoints the reference's
    ransac_voting_gpu.py produced for them (tests/golden/*_v3_512.npz; no
    oracle involved)."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from tests import golden_io as G
    res = {}
    for case in ("cat_v3_512", "synth_v3_512"):
        g = G.load(case)
        mask, vertex = (G.cat_inputs(g) if case.startswith("cat") else G.synth_inputs(g))[:2]
        kp = rvg.ransac_voting_layer_v3(torch.from_numpy(mask).to(dev), torch.from_numpy(vertex).to(dev), 512,
                                        _idxs=g["idxs"]).cpu().numpy()
        l2 = np.linalg.norm(kp - g["keypoints"], axis=-1)
        res[case.split("_")[0]] = dict(max_px=float(l2.max()), mean_px=float(l2.mean()))
    return res


def host_cores():
    """Every host core this process may run on: the affinity mask, bounded by
    the cgroup CPU quota when one is set (a GPU box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(budget_s):
    """The oracle's v3 (C kernels, OpenMP) on the host cores, on a bounded
    sample of the same workload (S(1234), hn=512): every core this process
    may use (host_cores()) and one thread, each image timed, median reported."""
    from oracle import oracle as O
    from pvnet_amd import synth
    f = synth.synthetic_field(1234)
    mask = np.argmax(f["seg"], 1)
    vertex = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, H, W, VN, 2))
    orig = O.vote_counts

    def run(threads, budget, max_n):
        def vc(direct, coords, hyp, thr, nthreads=0):
            return orig(direct, coords, hyp, thr, nthreads=threads)
        O.vote_counts = vc
        times = []
        try:
            O.ransac_voting_layer_v3(mask, vertex, 512, seed=0)       # warm-up
            t_end = time.perf_counter() + budget
            while len(times) < max_n and (len(times) < 1 or time.perf_counter() < t_end):
                t0 = time.perf_counter()
                O.ransac_voting_layer_v3(mask, vertex, 512, seed=len(times) + 1)
                times.append(time.perf_counter() - t0)
        finally:
            O.vote_counts = orig
        return times

    threads = host_cores()
    tm = run(threads, budget_s * 0.6, 50)
    t1 = run(1, budget_s * 0.4, 5)
    return dict(value=round(1.0 / float(np.median(tm)), 3), unit="images/sec", cores=threads, kind="port",
                affinity_cpus=len(os.sched_getaffinity(0)),
                value_1core=round(1.0 / float(np.median(t1)), 4),
                sample=f"median of {len(tm)} ({threads} threads) / {len(t1)} (1 thread) S(1234) 480x640 fields, "
                       f"tn=29861, hn=512: v3 incl. compaction + refine (oracle/pvvote_oracle.c, OpenMP)")


def library_config():
    """The loaded HIP library: path, version and its compile-time kernel
    choices (pv_build_config) -- no environment variable selects kernels."""
    from pvnet_amd import _lib
    L = _lib.load()
    return dict(path=os.path.relpath(_lib.LIB_PATH, REPO), version=L.pv_version().decode(),
                build=L.pv_build_config().decode())


def report(args, ws, res, final_err, dev):
    K, M = args.steps, args.per_step
    elapsed = res["elapsed"]
    value = res["n_images"] / elapsed
    tn = res["tn"]
    vote_ms = float(np.mean(res["vote_ms"]))
    pairs = float(args.hn * VN * tn)                # per launch: one launch votes one batch-1 frame
    flops = 12.0 * pairs                            # 12 FLOP per (h,v,t)
    achieved = flops / (vote_ms * 1e-3) / 1e12
    vc = dict(bound="valu", kernel="k_vote_mfma (fused vote+count, U2)", achieved=round(achieved, 2),
              peak=FP32_VECTOR_PEAK_TFLOPS, unit="TFLOP/s", frac=round(achieved / FP32_VECTOR_PEAK_TFLOPS, 4),
              traffic=pmc_traffic("k_vote_mfma"), avg_kernel_ms=round(vote_ms, 5), flop_per_launch=flops,
              note="12 FLOP per (hypothesis, keypoint, pixel) pair (SURVEY 8(d) U2) against the f32 vector peak; "
                   "the kernel evaluates the pair's two linear forms on the matrix cores (f16 hi/lo split, "
                   "v_mfma_f32_32x32x8_f16) and keeps z, the sign count and the guard band on the VALU, which "
                   "bounds it; no inlier mask is materialised (compulsory bytes: the pixel operands, 16 B per "
                   "pixel and keypoint, and the counts); traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (%s); "
                   "avg_kernel_ms from hipEvents the library records around the kernel on its stream in eager "
                   "calls (rocprof durations of the same run: %s)" % (PMC_FILE, STATS_FILE))
    # U3: argmax + compaction + strided gather of one frame,
    # HBM-read bound: H*W*(2 + 2K)*4 B read + tn*(2K + 2)*4 B written
    comp_ms = float(np.mean(res["compact_ms"]))
    u3_bytes = H * W * (2 + 2 * VN) * 4 + tn * (2 * VN + 2) * 4
    u3_gbs = u3_bytes / (comp_ms * 1e-3) / 1e9
    tc = [pmc_traffic(k) for k in ("k_fg_count", "k_compact")]
    rc = dict(bound="hbm", kernel="k_fg_count + k_compact (U3: seg_pred argmax, compaction, vertex gather)",
              achieved=round(u3_gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(u3_gbs / HBM_PEAK_GBS, 4),
              traffic=None if None in tc else int(sum(tc)), avg_kernel_ms=round(comp_ms, 5),
              bytes_per_launch=int(u3_bytes),
              note="algorithmic bytes H*W*(2+2K)*4 + tn*(2K+2)*4 (SURVEY 8(d) U3) / the two kernels' time "
                   "between an event recorded before the call and the library's ev_compact_end, eager calls "
                   "(launch gaps included); the pipeline writes 16 B per pixel and keypoint (the reference's "
                   "(cx, cy, nx, ny) operands), not 8; since round 6 the k_compact launch also makes the "
                   "frame's hypotheses (its first blocks, PVV_HYPFUSE), so this time includes that work (U2's "
                   "input, not U3's bytes); traffic = the two kernels' PMC bytes (%s)" % PMC_FILE)
    line = {
        "metric": "images/sec (480x640, 9 kp) vote->keypoint",
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": ws,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic S(seed) fields (SURVEY 8(d)): disk r=97.5 -> 29,861 fg px, 9 kp, 0.05 rad noise, "
                "20%% outliers; network-layout seg_pred/vertex_pred f32 resident in HBM, %d distinct fields per "
                "GPU cycled (%.0f MB, beyond the 256 MiB Infinity Cache)" % (args.fields, args.fields * 24.576),
        "config": {"workload": "stream of LINEMOD-cat-sized batch-1 frames (configs[1]'s voting layer): "
                               "ransac_voting_layer_v3 (hn=%d, thr=0.99) from seg_pred/vertex_pred; one step = one "
                               "hipGraph replay voting %d frames per GPU, %d in flight on separate streams; "
                               "images sharded round-robin over ranks, one gather of all keypoints at the end"
                               % (args.hn, M, max(1, args.inflight)),
                   "global_batch": M * ws, "per_gpu_batch_per_step": M, "image": [H, W], "keypoints": VN,
                   "round_hyp_num": args.hn, "foreground_px": int(tn),
                   "parallelism": "dp%d (images sharded round-robin, RCCL all_gather of keypoints)" % ws,
                   "images_in_flight": max(1, args.inflight), "stream_images": res["n_images"]},
        "roofline": None,
        "roofline_vote_count": vc,
        "roofline_compaction": rc,
        "max_kp_err_px": round(final_err, 5),
        "stream_order_max_err_px": round(res["order_err"], 5),
        "stream_order_ok": res["order_err"] <= 5.0,
        "latency_ms_per_image": round(res["latency_ms"], 5),
        "host_ms_per_replay": round(res["host_ms_per_replay"], 4),
        "kernel_nodes_per_frame": kernel_nodes(1, args.hn),
        "rank_cpus": args.rank_cpus_all,
        "rank_cpus_source": args.rank_cpus[1],
        "library": library_config(),
    }
    if res.get("batched") is not None:
        line["stream_batched4"] = res["batched"]
    if res.get("config3") is not None:
        line["stream_config3"] = res["config3"]
    if res.get("config4") is not None:
        line["stream_config4"] = res["config4"]
    try:
        line["kp_err_vs_ref_px"] = measure_kp_vs_ref(dev)
    except Exception as e:
        line["kp_err_vs_ref_px"] = {"error": repr(e)}
    # `roofline`: the kernel the north star names, voting_for_hypothesis (U1),
    # against the HBM peak; the pipeline's own dominant kernel (k_vote_mfma,
    # VALU-bound: no inlier mask is materialised) is `roofline_vote_count`,
    # its compaction (U3) `roofline_compaction`
    if not args.skip_u1:
        try:
            u1 = measure_u1(dev, args.hn)
            line["roofline"] = dict(bound="hbm", kernel=u1["kernel"], achieved=round(u1["achieved_gbs"], 1),
                                    peak=HBM_PEAK_GBS, unit="GB/s", frac=round(u1["frac"], 4),
                                    traffic=u1["traffic"], avg_kernel_ms=round(u1["ms"], 5),
                                    bytes_per_launch=u1["bytes_per_launch"], hn=u1["hn"], tn=u1["tn"],
                                    note="algorithmic bytes 8*tn*vn + 8*tn + 8*hn*vn + hn*vn*tn (SURVEY 8(d) U1) "
                                         "per launch / avg_kernel_ms = hipEvents around 3 replays of a hipGraph of 100 "
                                         "calls on the launching stream, queued behind 5 untimed replays (sustained "
                                         "steady state: each launch's writes drain behind the next); rocprof kernel "
                                         "durations of "
                                         "the same command: %s; "
                                         "traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (%s)" % (STATS_FILE, PMC_FILE))
        except Exception as e:  # reported, never hides the main number
            line["roofline"] = {"error": repr(e)}
    if not args.skip_u4:
        try:
            line["roofline_evd"] = measure_u4(dev)
        except Exception as e:  # reported, never hides the main number
            line["roofline_evd"] = {"error": repr(e)}
    if not args.skip_e2e:
        for key, fn in (("e2e_config1", lambda: measure_e2e(dev)),
                        ("e2e_config2_fp16_batch32", lambda: measure_e2e(dev, half=True, batch=32)),
                        ("voting_config2_batch32", lambda: measure_batch(dev)),
                        ("pnp_config5", lambda: measure_pnp(dev)),
                        ("pose_config5_batch32", lambda: measure_pose(dev)),
                        ("e2e_config4_fp16_batch32", lambda: measure_e2e_config4(dev))):
            try:
                line[key] = fn()
            except Exception as e:
                line[key] = {"error": repr(e)}
    if not args.skip_cpu:       # rank 0, at every N (the other ranks wait at the final barrier)
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    assert line["n_gpus"] == args.gpus, (line["n_gpus"], args.gpus)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
