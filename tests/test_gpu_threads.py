"""Concurrent callers: the reference's layers are called
from DataParallel worker threads at once, one per GPU, each on torch's
current stream of its device (/root/reference/tools/parallel.py:183-200,
tools/demo.py:174, tools/train_linemod.py:222-223).  On one MI355X the
analogue is several host threads, each launching on its own stream with its
own workspace.  Here two threads on cuda:0:

  * run eager v3 (int64 mask + strided vertex view, and the fused network
    layout) and EVD-with-mean calls at the same time, then
  * replay separately captured graphs of the same calls at the same time --
    graphs captured on their own streams with explicit workspaces, and graphs
    captured on torch's one shared capture stream with the default workspace
    (each capture then owns its scratch);

every result is bit-equal to the single-thread result and matches the golden
fixtures.  Plus: a workspace handed to a second stream while a call on the
first is in flight is refused, streams from pvnet_amd.streams are distinct
(torch.cuda.Stream() wraps round a pool of 32), and two graphs of split-K
convolutions captured on one shared stream replay concurrently without
sharing arrival counters."""
import threading

import numpy as np
import pytest
import torch

from pvnet_amd import streams
from tests import golden_io as G

pytestmark = pytest.mark.gpu

KP_TOL = 1e-2
COV_RTOL = 1e-4
REPS = 6            # eager rounds per thread
REPLAYS = 12        # concurrent replays per thread


def cu(x, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t.to(dev) if dtype is None else t.to(device=dev, dtype=dtype)


@pytest.fixture(scope="module")
def rvg():
    from pvnet_amd import ransac_voting_gpu
    return ransac_voting_gpu


@pytest.fixture(scope="module")
def cases(device):
    """Device inputs and golden results of three calls: v3 on LINEMOD 'cat'
    (int64 mask, strided view), v3 from the network layout on S(1234), and
    EVD with mean on S(1234)."""
    gc = G.load("cat_v3_512")
    mc, vc, _ = G.cat_inputs(gc)
    gs = G.load("synth_v3_512")
    _, _, fs = G.synth_inputs(gs)
    ge = G.load("synth_evdm")
    me, ve, _ = G.synth_inputs(ge)
    i32 = torch.int32      # device-resident pixel pairs: nothing is copied inside a capture
    return dict(
        cat=(cu(mc, device), cu(vc, device), cu(gc["idxs"], device, i32), gc["keypoints"]),
        net=(cu(fs["seg"], device), cu(fs["vertex"], device), cu(gs["idxs"], device, i32), gs["keypoints"]),
        evd=(cu(me, device), cu(ve, device), cu(ge["idxs"][0].reshape(1, -1, 9, 2), device, i32),
             cu(ge["mean"], device), ge["cov"]))


def run_calls(rvg, cases, ws, out):
    """The three calls on the current stream with workspaces ws[0..2],
    results into out (kp_cat [1,9,2], kp_net [1,9,2], cov [1,9,2,2])."""
    m, v, idxs, _ = cases["cat"]
    out[0].copy_(rvg.ransac_voting_layer_v3(m, v, 512, _idxs=idxs, _workspace=ws[0]))
    s, ver, idxs, _ = cases["net"]
    rvg.ransac_voting_layer_v3_from_network(s, ver, 512, _idxs=idxs, _workspace=ws[1], out=out[1])
    m, v, idxs, mean, _ = cases["evd"]
    out[2].copy_(rvg.estimate_voting_distribution_with_mean(m, v, mean, _idxs=idxs, _workspace=ws[2])[1])


def new_out(device):
    return [torch.zeros((1, 9, 2), device=device), torch.zeros((1, 9, 2), device=device),
            torch.zeros((1, 9, 2, 2), device=device)]


def check_golden(cases, res):
    np.testing.assert_allclose(res[0], cases["cat"][3], atol=KP_TOL, rtol=0)
    np.testing.assert_allclose(res[1], cases["net"][3], atol=KP_TOL, rtol=0)
    gcov = cases["evd"][4]
    np.testing.assert_allclose(res[2], gcov, rtol=COV_RTOL, atol=1e-4 * np.abs(gcov).max())


def run_threads(fn, n=2):
    """fn(i) in n threads at once; re-raises the first failure."""
    errs = [None] * n

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:   # noqa: BLE001 -- handed to the main thread
            errs[i] = e
    th = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a worker thread hung"
    for e in errs:
        if e is not None:
            raise e


def test_two_threads_eager_and_replays_bit_equal(device, rvg, cases):
    torch.cuda.set_device(device)
    # single-thread reference results (their own stream and workspaces)
    s0 = streams.new_stream(device)
    ref_out = new_out(device)
    with torch.cuda.stream(s0):
        run_calls(rvg, cases, [rvg.VotingWorkspace() for _ in range(3)], ref_out)
    s0.synchronize()
    ref = [o.cpu().numpy() for o in ref_out]
    check_golden(cases, ref)

    n = 2
    lanes = [streams.new_stream(device) for _ in range(n)]
    assert len({s.cuda_stream for s in lanes + [s0]}) == n + 1
    works = [[rvg.VotingWorkspace() for _ in range(3)] for _ in range(n)]
    eager = [[] for _ in range(n)]
    go = threading.Barrier(n)

    # phase 1: eager calls from both threads at once, REPS rounds each
    def eager_phase(i):
        torch.cuda.set_device(device)
        go.wait()
        with torch.cuda.stream(lanes[i]):
            for _ in range(REPS):
                o = new_out(device)
                run_calls(rvg, cases, works[i], o)
                eager[i].append(o)
        lanes[i].synchronize()
    run_threads(eager_phase, n)
    for i in range(n):
        for o in eager[i]:
            for k in range(3):
                np.testing.assert_array_equal(o[k].cpu().numpy(), ref[k], err_msg=f"thread {i} eager call {k}")

    # phase 2: each thread captures its own graph (one capture at a time),
    # then both replay at once; two kinds of graph per thread:
    #   own  -- captured on the thread's stream with its explicit workspaces
    #   dflt -- captured on torch.cuda.graph's shared capture stream with the
    #           default workspace (each capture takes its own scratch)
    cap_lock = threading.Lock()
    graphs = [dict() for _ in range(n)]
    gouts = [dict(own=new_out(device), dflt=new_out(device)) for _ in range(n)]
    cap_done = threading.Barrier(n)

    def graph_phase(i):
        torch.cuda.set_device(device)
        with cap_lock:
            g_own, g_dflt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.stream(lanes[i]):
                with torch.cuda.graph(g_own, stream=lanes[i]):
                    run_calls(rvg, cases, works[i], gouts[i]["own"])
            with torch.cuda.graph(g_dflt):
                run_calls(rvg, cases, [None, None, None], gouts[i]["dflt"])
            torch.cuda.synchronize()
            graphs[i] = dict(own=g_own, dflt=g_dflt)
        cap_done.wait()
        results = []
        with torch.cuda.stream(lanes[i]):
            for r in range(REPLAYS):
                for kind in ("own", "dflt"):
                    for o in gouts[i][kind]:
                        o.zero_()
                    graphs[i][kind].replay()
                    results.append((kind, [o.clone() for o in gouts[i][kind]]))
        lanes[i].synchronize()
        graphs[i]["results"] = results
    run_threads(graph_phase, n)
    for i in range(n):
        assert len(graphs[i]["results"]) == 2 * REPLAYS
        for kind, o in graphs[i]["results"]:
            for k in range(3):
                np.testing.assert_array_equal(o[k].cpu().numpy(), ref[k], err_msg=f"thread {i} {kind} replay {k}")
    check_golden(cases, [o.cpu().numpy() for o in graphs[0]["results"][-1][1]])


def test_workspace_refuses_second_stream_in_flight(device, rvg, cases):
    """An explicit workspace whose call on stream A is still queued (behind a
    device sleep) is refused on stream B; once A has drained it moves to B."""
    torch.cuda.set_device(device)
    a, b = streams.new_stream(device), streams.new_stream(device)
    ws = rvg.VotingWorkspace()
    s, ver, idxs, kp = cases["net"]
    out = torch.zeros((1, 9, 2), device=device)
    with torch.cuda.stream(a):
        rvg.ransac_voting_layer_v3_from_network(s, ver, 512, _idxs=idxs, _workspace=ws, out=out)
    a.synchronize()
    with torch.cuda.stream(a):
        torch.cuda._sleep(200_000_000)     # ~0.1 s of device clocks ahead of the call
        rvg.ransac_voting_layer_v3_from_network(s, ver, 512, _idxs=idxs, _workspace=ws, out=out)
    with torch.cuda.stream(b):
        with pytest.raises(RuntimeError, match="in flight on another stream"):
            rvg.ransac_voting_layer_v3_from_network(s, ver, 512, _idxs=idxs, _workspace=ws, out=out)
    a.synchronize()
    out2 = torch.zeros_like(out)
    with torch.cuda.stream(b):
        rvg.ransac_voting_layer_v3_from_network(s, ver, 512, _idxs=idxs, _workspace=ws, out=out2)
    b.synchronize()
    assert torch.equal(out, out2)
    np.testing.assert_allclose(out2.cpu().numpy(), kp, atol=KP_TOL, rtol=0)


def test_streams_are_distinct_torch_pool_wraps(device):
    """pvnet_amd.streams.new_stream creates real streams (40 distinct
    handles); torch.cuda.Stream() hands out a pool of 32 per priority, so 40
    of those hold at most 32 distinct handles (the reason the library's
    lanes and the bench take theirs from new_stream)."""
    ours = [streams.new_stream(device) for _ in range(40)]
    assert len({s.cuda_stream for s in ours}) == 40
    pooled = [torch.cuda.Stream(device=device) for _ in range(40)]
    assert len({s.cuda_stream for s in pooled}) <= 32
    # capture ids: 0 outside a capture, the same id on a lane forked into it
    assert streams.capture_id(ours[0]) == 0
    g = torch.cuda.CUDAGraph()
    x = torch.zeros(4, device=device)
    with torch.cuda.stream(ours[0]):
        with torch.cuda.graph(g, stream=ours[0]):
            cid = streams.capture_id()
            ours[1].wait_stream(ours[0])
            with torch.cuda.stream(ours[1]):
                x.add_(1)
                cid1 = streams.capture_id()
            ours[0].wait_stream(ours[1])
    assert cid != 0 and cid1 == cid
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(x, torch.ones(4, device=device))


def test_two_threads_split_conv_graphs_shared_capture_stream(device):
    """Two graphs of one split-K convolution (pv_conv3x3_ex_f16's last round
    cut in parts, arrival counters in its scratch), both captured on
    torch.cuda.graph's shared capture stream, replayed at once from two
    threads on their own streams: each capture owns its scratch and zeroes
    its counters, so every replay equals the eager result bit for bit."""
    from pvnet_amd import _lib
    from pvnet_amd.network import conv3x3, conv3x3_weight
    torch.cuda.set_device(device)
    g = torch.Generator().manual_seed(505)
    cl = torch.channels_last
    n, cin, cout, h, w = 16, 128, 128, 60, 80
    need = _lib.load().pv_conv3x3_workspace_bytes(n * h * w, cout, 9 * cin // 64)
    assert need > 0, "the case must take the split-K path"
    xs = [torch.randn(n, cin, h, w, generator=g).to(device, torch.float16).contiguous(memory_format=cl)
          for _ in range(2)]
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1, bias=True)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5))
        conv.bias.copy_(torch.randn(cout, generator=g) * 0.5)
    conv = conv.to(device).half()
    wt = conv3x3_weight(conv)
    with torch.no_grad():
        ref = [conv3x3(x, wt, conv.bias, 1, "relu") for x in xs]
    torch.cuda.synchronize()
    outs, graphs = [None, None], [None, None]
    for i in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(gr):
            outs[i] = conv3x3(xs[i], wt, conv.bias, 1, "relu")
        graphs[i] = gr
    torch.cuda.synchronize()
    lanes = [streams.new_stream(device) for _ in range(2)]
    got = [[], []]
    go = threading.Barrier(2)

    def replay(i):
        torch.cuda.set_device(device)
        go.wait()
        with torch.cuda.stream(lanes[i]):
            for _ in range(REPLAYS):
                outs[i].zero_()
                graphs[i].replay()
                got[i].append(outs[i].clone())
        lanes[i].synchronize()
    run_threads(replay, 2)
    for i in range(2):
        for o in got[i]:
            assert torch.equal(o, ref[i])


_RELEASE_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, %r)
from pvnet_amd import streams, ransac_voting_gpu as rvg
from tests import golden_io as G
gs = G.load("synth_v3_512")
_, _, fs = G.synth_inputs(gs)
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
seg, ver = torch.from_numpy(fs["seg"]).to(dev), torch.from_numpy(fs["vertex"]).to(dev)
idxs = torch.from_numpy(np.ascontiguousarray(gs["idxs"])).to(dev, torch.int32)
res = []
for r in range(3):
    st = streams.new_stream(dev)
    ws = rvg.VotingWorkspace()
    out = torch.zeros((1, 9, 2), device=dev)
    with torch.cuda.stream(st):
        rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _idxs=idxs, _workspace=ws, out=out)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _idxs=idxs, _workspace=ws, out=out)
        out.zero_()
        g.replay()
    st.synchronize()
    res.append(out.cpu().numpy().copy())
    del g, ws
    streams.release(st, destroy=(r != 1))
assert streams.live_count() == 0
assert all(np.array_equal(res[0], x) for x in res[1:]), "results differ across re-created streams"
np.testing.assert_allclose(res[0], gs["keypoints"], atol=1e-2, rtol=0)
print("release-cycle ok", flush=True)
"""


def test_streams_release_recreate_bit_equal_exit_zero():
    """pvnet_amd.streams.release: a process creates a stream,
    votes on it eagerly and through a graph captured on it, drops the graph
    and workspace, releases the stream (destroyed twice, kept for reuse once)
    and creates the next; all three rounds bit-equal and within the golden
    tolerance, nothing left live, and the process exits 0 (round 5's exit
    crash came from streams destroyed at interpreter exit)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-X", "faulthandler", "-c", _RELEASE_CHILD % repo], cwd=repo,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, f"exit {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
    assert "release-cycle ok" in p.stdout
