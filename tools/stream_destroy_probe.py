"""Which use of a destroyed HIP stream crashes a process (round-5 exit crash,
DESIGN.md 2a).  Each case runs in a child process of its own (faulthandler
on) and the parent prints the child's exit status and the last lines of its
stderr.  GPU only; a diagnostic, not part of the product or the tests.

    python tools/stream_destroy_probe.py            # every case
    python tools/stream_destroy_probe.py <case>     # one case, in this process

Cases (a stream from pv_stream_create, destroyed with pv_stream_destroy):
  plain        launch, synchronize, destroy, exit
  graph_alive  capture a graph on the stream, destroy the stream, replay the graph, drop it, exit
  rec_free     tensor.record_stream(stream), destroy the stream, then free the tensor (the
               caching allocator records its reuse event on the dead stream)
  rec_exit     as rec_free but the tensor is a module global freed at interpreter teardown,
               the stream destroyed by a weakref.finalize at exit (round 5's form)
  release      pvnet_amd.streams.release() after the stream's uses are gone, re-create, exit
"""
import subprocess
import sys

CASES = ["plain", "graph_alive", "rec_free", "rec_exit", "release"]


def child(case):
    import ctypes
    import faulthandler
    import weakref
    faulthandler.enable()
    import torch
    sys.path.insert(0, ".")
    from pvnet_amd import _lib, streams
    L = _lib.load()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)

    def make():
        h = ctypes.c_void_p()
        _lib.check(L.pv_stream_create(0, ctypes.byref(h)), "create")
        return h.value, torch.cuda.ExternalStream(h.value, device=dev)

    x = torch.ones(1 << 20, device=dev)
    if case == "plain":
        h, st = make()
        with torch.cuda.stream(st):
            x.mul_(2)
        st.synchronize()
        _lib.check(L.pv_stream_destroy(h), "destroy")
    elif case == "graph_alive":
        h, st = make()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            x.mul_(1)
            with torch.cuda.graph(g, stream=st):
                x.mul_(1)
        st.synchronize()
        _lib.check(L.pv_stream_destroy(h), "destroy")
        g.replay()
        torch.cuda.synchronize()
        del g
    elif case == "rec_free":
        h, st = make()
        y = torch.empty(1 << 20, device=dev)
        with torch.cuda.stream(st):
            y.fill_(1)
        y.record_stream(st)
        st.synchronize()
        _lib.check(L.pv_stream_destroy(h), "destroy")
        del y
        torch.cuda.synchronize()
        print("freed", flush=True)
    elif case == "rec_exit":
        h, st = make()
        global KEEP
        KEEP = torch.empty(1 << 20, device=dev)
        with torch.cuda.stream(st):
            KEEP.fill_(1)
        KEEP.record_stream(st)
        weakref.finalize(st, L.pv_stream_destroy, h)
        globals()["ST"] = st
    elif case == "release":
        outs = []
        for r in range(3):
            st = streams.new_stream(dev)
            y = torch.empty(1 << 20, device=dev)
            with torch.cuda.stream(st):
                y.copy_(x).mul_(3)
            outs.append(y.sum().item())
            streams.release(st)
        print("release sums", outs, "live", streams.live_count(), flush=True)
    torch.cuda.synchronize()
    print("case", case, "body done", flush=True)


def main():
    if len(sys.argv) > 1:
        return child(sys.argv[1])
    for c in CASES:
        try:
            p = subprocess.run([sys.executable, __file__, c], capture_output=True, text=True, timeout=120)
            rc, tail = p.returncode, (p.stdout + p.stderr).strip().splitlines()[-8:]
        except subprocess.TimeoutExpired:
            rc, tail = "timeout", []
        print(f"== {c}: exit {rc}")
        for line in tail:
            print("   ", line)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
