"""HIP streams of their own, and the id of the capture a stream belongs to.

``torch.cuda.Stream()`` does not create a stream: it hands out one of 32
pooled streams per priority and device, round robin, so the 33rd "new"
stream is the 1st again (and every stream torch.cuda.graph captures on
without ``stream=`` is one shared side stream).  Two lanes, threads or
graphs that must not share a stream take theirs from :func:`new_stream`,
which creates a real one through libpvvote.so (``pv_stream_create``) and
wraps it as a ``torch.cuda.ExternalStream``.  Like torch's pooled streams
these live for the whole process (destroying them from a finalizer at
interpreter exit -- weakref.finalize's atexit pass -- crashed the process in
hipStreamDestroy on the GPU box): make one per lane or thread, once.

:func:`capture_id` is the id of the stream capture the current (or given)
stream belongs to, 0 outside a capture: scratch owned by one captured graph
(pvnet_amd.network's split-K counters) is keyed by it.

The reference's concurrent callers are DataParallel worker threads, one per
GPU, each launching on torch's current stream of its device
(/root/reference/tools/parallel.py:183-200); on one device the analogue is
one stream per launching thread.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_LIVE = []      # every stream made here, for the process's lifetime


def new_stream(device=None, priority: int = 0) -> torch.cuda.ExternalStream:
    """A non-blocking HIP stream nobody else launches on, on ``device``."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    L = _lib.load()
    h = ctypes.c_void_p()
    with torch.cuda.device(device):
        _lib.check(L.pv_stream_create(int(priority), ctypes.byref(h)), "pv_stream_create")
    st = torch.cuda.ExternalStream(h.value, device=device)
    _LIVE.append(st)
    return st


def capture_id(stream=None) -> int:
    """The capture id of ``stream`` (default: torch's current stream), 0 when
    it is not being captured."""
    if stream is None:
        stream = torch.cuda.current_stream()
    cid = ctypes.c_uint64(0)
    _lib.check(_lib.load().pv_stream_capture_id(stream.cuda_stream, ctypes.byref(cid)), "pv_stream_capture_id")
    return int(cid.value)
