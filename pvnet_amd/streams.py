"""HIP streams of their own, and the id of the capture a stream belongs to.

``torch.cuda.Stream()`` does not create a stream: it hands out one of 32
pooled streams per priority and device, round robin, so the 33rd "new"
stream is the 1st again (and every stream torch.cuda.graph captures on
without ``stream=`` is one shared side stream).  Two lanes, threads or
graphs that must not share a stream take theirs from :func:`new_stream`,
which creates a real one through libpvvote.so (``pv_stream_create``) and
wraps it as a ``torch.cuda.ExternalStream``.

Lifetime: :func:`release` hands a stream back once nothing will use it
again -- every graph captured on it dropped, every tensor that called
``record_stream`` on it freed (torch's caching allocator records a reuse
event on each such stream when the tensor is freed; on a destroyed stream
that is a call on a dead handle).  The stream is synchronized
and destroyed (``destroy=True``) or kept in a free list that the next
:func:`new_stream` of the same device and priority takes first.  Streams
still live at interpreter exit are not destroyed: the process's end
reclaims them, while a destroy from an atexit pass would run before the
module teardown frees the tensors that recorded them.

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
import threading

import torch

from . import _lib

_lock = threading.Lock()
_LIVE = {}      # handle -> (ExternalStream, device index, priority): handed out, not yet released
_FREE = {}      # (device index, priority) -> [ExternalStream]: released, kept for reuse


def new_stream(device=None, priority: int = 0) -> torch.cuda.ExternalStream:
    """A non-blocking HIP stream nobody else launches on, on ``device``."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _lock:
        free = _FREE.get((idx, int(priority)))
        if free:
            st = free.pop()
            _LIVE[st.cuda_stream] = (st, idx, int(priority))
            return st
    L = _lib.load()
    h = ctypes.c_void_p()
    with torch.cuda.device(idx):
        _lib.check(L.pv_stream_create(int(priority), ctypes.byref(h)), "pv_stream_create")
    st = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
    with _lock:
        _LIVE[h.value] = (st, idx, int(priority))
    return st


def release(stream: torch.cuda.ExternalStream, destroy: bool = True) -> None:
    """Give back a stream from :func:`new_stream`: waits for its work, then
    destroys it (``destroy=True``) or keeps it for the next :func:`new_stream`.
    The caller guarantees nothing uses it again: no graph captured on it is
    replayed afterwards and no tensor that ``record_stream``-ed it is still
    alive (free them, or pass ``destroy=False``)."""
    h = stream.cuda_stream
    with _lock:
        ent = _LIVE.get(h)
        if ent is None:
            raise ValueError("release(): not a live stream from pvnet_amd.streams.new_stream")
    if capture_id(stream) != 0:
        raise RuntimeError("release(): the stream is being captured")
    stream.synchronize()
    with _lock:
        _LIVE.pop(h, None)
        if not destroy:
            _FREE.setdefault((ent[1], ent[2]), []).append(stream)
            return
    with torch.cuda.device(ent[1]):
        _lib.check(_lib.load().pv_stream_destroy(h), "pv_stream_destroy")


def live_count() -> int:
    """Streams handed out by :func:`new_stream` and not released."""
    with _lock:
        return len(_LIVE)


def capture_id(stream=None) -> int:
    """The capture id of ``stream`` (default: torch's current stream), 0 when
    it is not being captured."""
    if stream is None:
        stream = torch.cuda.current_stream()
    cid = ctypes.c_uint64(0)
    _lib.check(_lib.load().pv_stream_capture_id(stream.cuda_stream, ctypes.byref(cid)), "pv_stream_capture_id")
    return int(cid.value)
