"""Drop-in for ``lib/ransac_voting_gpu_layer/ransac_voting_gpu.py`` (RV): the
voting layers the inference pipeline calls, with the reference's signatures.

``ransac_voting_layer_v3`` (RV:520-604) and
``estimate_voting_distribution_with_mean`` (RV:333-406) /
``estimate_voting_distribution`` (RV:263-331) run the whole batch on the
device in a fixed sequence of HIP kernels (libpvvote.so, one C-ABI call):
no per-image Python loop, no host synchronisation, graph-capturable.

Behaviour kept from the reference:
  * foreground = ``mask.byte() != 0`` for v3 (RV:533), ``mask == 1`` for EVD
    (RV:340); fewer than ``min_num`` pixels -> zeros (RV:537-540); more than
    ``max_num`` -> Bernoulli(max_num/fg) downsampling (RV:543-546);
  * row-major compaction, coords = (col, row) (RV:548-552);
  * ``idxs`` drawn once per call (RV:553): every iteration of the reference's
    ``while True`` loop re-creates the same hypotheses, so its best-so-far
    state is final after the first pass and the loop only repeats identical
    work (RV:558-582).  The device pipeline runs that pass once; the
    iteration count the loop would take is reported in ``_diag['iters']``;
  * first-index argmax, strict-greater best update (RV:568-575);
  * least squares on the winner's inliers with ``b_inv``'s batch-wide
    identity fallback when any keypoint's matrix is singular (RV:503-518).

Differences (documented in DESIGN.md): the random draws come from a counter
RNG seeded from torch's CPU generator, not from torch's device RNG (which
cannot be reproduced anyway); fp32 least-squares sums are accumulated in fp64
(the reference's fp32 order is unspecified).
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib

__all__ = ["ransac_voting_layer_v3", "ransac_voting_layer_v5", "ransac_motion_voting",
           "estimate_voting_distribution_with_mean",
           "estimate_voting_distribution",
           "b_inv", "ransac_voting_layer_v3_from_network", "VotingWorkspace"]

_MASK_KIND = {torch.int64: _lib.PV_MASK_I64, torch.uint8: _lib.PV_MASK_U8, torch.bool: _lib.PV_MASK_U8,
              torch.int32: _lib.PV_MASK_I32}
_SEG_KIND = {torch.float32: _lib.PV_MASK_SEG_F32, torch.float16: _lib.PV_MASK_SEG_F16}
_VERTEX_KIND = {torch.float32: _lib.PV_VERTEX_F32, torch.float16: _lib.PV_VERTEX_F16}


def _draw_seed() -> int:
    # torch's default CPU generator: reproducible under torch.manual_seed, no device sync
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class VotingWorkspace:
    """Device scratch for the pipelines, reused across calls of the same shape
    (needed for hipGraph capture: no allocation inside the captured region).

    A pipeline call zeroes and rewrites its workspace, so two calls in flight
    on different streams must not share one.

    * An explicit workspace (``_workspace=``, ``per_stream=False``) holds one
      call at a time: an eager call on a stream other than the one its
      previous call ran on raises ``RuntimeError`` if that call is still in
      flight (an event recorded after each call), so two threads handing one
      workspace to their own streams get an error, not a race.  The check is
      host-side: it cannot see a ``wait_stream`` that orders the two streams,
      so a caller that orders them itself passes ``check_streams=False``.
      Inside a
      graph capture there is no check (the call runs when the graph is
      replayed): a workspace captured into a graph belongs to that graph, and
      two graphs that may replay at the same time need one each.  Growing
      inside a capture raises: warm the workspace up (one eager call of the
      same shape) before capturing.
    * The default workspace (used when ``_workspace`` is omitted,
      ``per_stream=True``) keeps one buffer per (device, stream) for eager
      calls, and inside a capture takes a fresh buffer from the capturing
      graph's private memory pool for every call: each captured graph owns
      its scratch, so graphs captured on one shared stream (torch.cuda.graph
      without ``stream=``) can replay concurrently.

    A buffer that grows is released with ``record_stream`` for every stream
    that used it, so the caching allocator never hands it out while a kernel
    can still touch it.  Thread-safe (one lock per workspace)."""

    def __init__(self, per_stream: bool = False, check_streams: bool = True):
        self._buf = {}
        self._streams = {}
        self._per_stream = per_stream
        self._check = check_streams
        self._lock = threading.Lock()
        self._owner = {}       # explicit: key -> [stream handle of the last call, busy, event after it]

    def _key(self, device, stream):
        return (str(device), stream.cuda_stream) if self._per_stream else (str(device),)

    def get(self, device, nbytes: int) -> torch.Tensor:
        stream = torch.cuda.current_stream(device)
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing and self._per_stream:
            # the default workspace inside a capture: the graph's own (private pool)
            return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        key = self._key(device, stream)
        with self._lock:
            own = None
            if not self._per_stream and not capturing:
                own = self._owner.setdefault(key, [stream.cuda_stream, False, None])
                if self._check and own[0] != stream.cuda_stream and \
                        (own[1] or (own[2] is not None and not own[2].query())):
                    raise RuntimeError("VotingWorkspace is in use by a call in flight on another stream: give each "
                                       "stream (each launching thread) its own workspace")
            buf = self._buf.get(key)
            if buf is None or buf.numel() < nbytes:
                if capturing:
                    raise RuntimeError("VotingWorkspace would allocate during graph capture: make one eager call of "
                                       "the same shape with this workspace (_workspace=...) before capturing")
                if buf is not None:
                    for st in self._streams.get(key, ()):
                        buf.record_stream(st)
                buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
                self._buf[key] = buf
                self._streams[key] = set()
            self._streams[key].add(stream)
            if own is not None:
                # busy only once the buffer is in hand: a failed allocation leaves the workspace free
                own[0], own[1] = stream.cuda_stream, True
            return buf

    def done(self, device) -> None:
        """After the library call that used get()'s buffer was queued (or
        failed): an event on its stream marks when the workspace is free."""
        if self._per_stream or torch.cuda.is_current_stream_capturing():
            return
        stream = torch.cuda.current_stream(device)
        with self._lock:
            own = self._owner.get(self._key(device, stream))
            if own is None or own[0] != stream.cuda_stream:
                return
            if own[2] is None:
                own[2] = torch.cuda.Event()
            own[2].record(stream)
            own[1] = False


_default_ws = VotingWorkspace(per_stream=True)


def _desc(mask, vertex, seg=False):
    if not (isinstance(vertex, torch.Tensor) and vertex.is_cuda):
        raise RuntimeError("vertex must be a CUDA tensor")
    if not (isinstance(mask, torch.Tensor) and mask.is_cuda):
        raise RuntimeError("mask must be a CUDA tensor")
    if vertex.dim() != 5 or vertex.shape[4] != 2:
        raise RuntimeError("vertex must be [b,h,w,vn,2]")
    b, h, w, vn, _ = vertex.shape
    if vertex.dtype not in _VERTEX_KIND:
        raise RuntimeError(f"vertex dtype {vertex.dtype} not supported (float32/float16)")
    if mask.device != vertex.device:
        raise RuntimeError("mask and vertex must be on the same device")
    d = _lib.ImageDesc()
    d.mask = mask.data_ptr()
    if seg:
        if mask.dim() != 4 or mask.shape[1] != 2 or tuple(mask.shape[2:]) != (h, w) or mask.shape[0] != b:
            raise RuntimeError("seg_pred must be [b,2,h,w]")
        if mask.dtype not in _SEG_KIND:
            raise RuntimeError(f"seg_pred dtype {mask.dtype} not supported")
        d.mask_kind = _SEG_KIND[mask.dtype]
        for i in range(4):
            d.mask_strides[i] = mask.stride(i)
    else:
        if tuple(mask.shape) != (b, h, w):
            raise RuntimeError(f"mask must be [b,h,w] = {(b, h, w)}, got {tuple(mask.shape)}")
        if mask.dtype not in _MASK_KIND:
            raise RuntimeError(f"mask dtype {mask.dtype} not supported")
        d.mask_kind = _MASK_KIND[mask.dtype]
        for i in range(3):
            d.mask_strides[i] = mask.stride(i)
    d.vertex = vertex.data_ptr()
    d.vertex_kind = _VERTEX_KIND[vertex.dtype]
    for i in range(5):
        d.vertex_strides[i] = vertex.stride(i)
    d.b, d.H, d.W, d.vn = b, h, w, vn
    return d


def _params(round_hyp_num, inlier_thresh, confidence=0.99, max_iter=100, min_num=100, max_num=30000, seed=None,
            idxs=None, keep=None, min_hyp_num=0, topk=0):
    p = _lib.VoteParams()
    p.round_hyp_num = int(round_hyp_num)
    p.inlier_thresh = float(inlier_thresh)
    p.confidence = float(confidence)
    p.max_iter = int(max_iter)
    p.min_num = int(min_num)
    p.max_num = int(max_num)
    p.seed = _draw_seed() if seed is None else int(seed) & (2 ** 64 - 1)
    p.idxs = idxs.data_ptr() if idxs is not None else None
    p.keep = keep.data_ptr() if keep is not None else None
    p.min_hyp_num = int(min_hyp_num)
    p.topk = int(topk)
    return p


def _aux(x, dtype, device, shape, name):
    if x is None:
        return None
    x = torch.as_tensor(x).to(device=device, dtype=dtype).contiguous()
    if tuple(x.shape) != tuple(shape):
        raise RuntimeError(f"{name} must have shape {tuple(shape)}, got {tuple(x.shape)}")
    return x


def _v3(d, mask, vertex, round_hyp_num, inlier_thresh, confidence, max_iter, min_num, max_num, _idxs, _keep, _diag,
        _seed, _workspace, out=None, conf_thresh=None):
    dev = vertex.device
    b, h, w, vn = d.b, d.H, d.W, d.vn
    idxs = _aux(_idxs, torch.int32, dev, (b, round_hyp_num, vn, 2), "_idxs")
    keep = _aux(_keep, torch.uint8, dev, (b, h, w), "_keep")
    prm = _params(round_hyp_num, inlier_thresh, confidence, max_iter, min_num, max_num, _seed, idxs, keep)
    L = _lib.load()
    nbytes = L.pv_v3_workspace_size(b, h, w, vn, round_hyp_num)
    work = _workspace or _default_ws
    if out is None:
        out = torch.empty((b, vn, 2), dtype=torch.float32, device=dev)
    diag = None
    dt = {}
    if _diag is not None:
        dt = dict(hyp=torch.empty((b, round_hyp_num, vn, 2), dtype=torch.float32, device=dev),
                  counts=torch.empty((b, vn, round_hyp_num), dtype=torch.int32, device=dev),
                  win_idx=torch.empty((b, vn), dtype=torch.int32, device=dev),
                  win_ratio=torch.empty((b, vn), dtype=torch.float32, device=dev),
                  tn=torch.empty((b,), dtype=torch.int32, device=dev),
                  iters=torch.empty((b,), dtype=torch.int32, device=dev),
                  ata=torch.empty((b, vn, 2, 2), dtype=torch.float32, device=dev),
                  atb=torch.empty((b, vn, 2), dtype=torch.float32, device=dev))
        diag = _lib.V3Diag(**{k: v.data_ptr() for k, v in dt.items()})
    conf = None if conf_thresh is None else torch.empty((b, vn), dtype=torch.float32, device=dev)
    ws = work.get(dev, nbytes)
    with torch.cuda.device(dev):
        try:
            if conf_thresh is None:
                code = L.pv_ransac_voting_v3(ctypes.byref(d), ctypes.byref(prm), out.data_ptr(), ws.data_ptr(), nbytes,
                                             ctypes.byref(diag) if diag is not None else None,
                                             torch.cuda.current_stream(dev).cuda_stream)
            else:
                code = L.pv_ransac_voting_v5(ctypes.byref(d), ctypes.byref(prm), float(conf_thresh), out.data_ptr(),
                                             conf.data_ptr(), ws.data_ptr(), nbytes,
                                             ctypes.byref(diag) if diag is not None else None,
                                             torch.cuda.current_stream(dev).cuda_stream)
        finally:
            work.done(dev)
    _lib.check(code, "ransac_voting_layer_v3" if conf_thresh is None else "ransac_voting_layer_v5")
    if _diag is not None:
        _diag.update(dt)
    # keep the inputs alive until the kernels that read them have been queued
    del mask, idxs, keep
    return out if conf is None else (out, conf)


def ransac_voting_layer_v3(mask, vertex, round_hyp_num, inlier_thresh=0.99, confidence=0.99, max_iter=100,
                           min_num=100, max_num=30000, *, _idxs=None, _keep=None, _diag=None, _seed=None,
                           _workspace=None):
    """RV:520-604.  mask [b,h,w] (int64/int32/uint8/bool), vertex [b,h,w,vn,2]
    (f32 or f16, any strides -- e.g. the permuted view of vertex_pred) ->
    f32 [b,vn,2] on the same device.

    Test hooks (keyword-only, not in the reference): ``_idxs`` [b,hn,vn,2]
    pixel pairs instead of the RNG, ``_keep`` [b,h,w] downsampling mask,
    ``_diag`` dict filled with intermediate device tensors, ``_seed``."""
    d = _desc(mask, vertex)
    return _v3(d, mask, vertex, round_hyp_num, inlier_thresh, confidence, max_iter, min_num, max_num, _idxs,
               _keep, _diag, _seed, _workspace)


def ransac_voting_layer_v5(mask, vertex, round_hyp_num, inlier_thresh=0.999, confidence=0.99, max_iter=20,
                           min_num=5, max_num=100, *, _idxs=None, _keep=None, _diag=None, _seed=None,
                           _workspace=None):
    """RV:769-864 (the uncertainty eval wrapper's layer, TRAIN:123): v3 with
    v5's defaults, returning (points f32 [b,vn,2], confidence f32 [b,vn]) --
    each refined keypoint's inlier ratio at 0.999 (RV:856-858)."""
    d = _desc(mask, vertex)
    return _v3(d, mask, vertex, round_hyp_num, inlier_thresh, confidence, max_iter, min_num, max_num, _idxs,
               _keep, _diag, _seed, _workspace, conf_thresh=0.999)


def ransac_motion_voting(mask, vertex):
    """RV:966-987: mask [b,h,w], vertex [b,h,w,vn,2] holding offsets ->
    f32 [b,vn,2], the foreground mean of vertex + (col, row) (zeros for an
    empty mask), in one HIP kernel."""
    d = _desc(mask, vertex)
    out = torch.empty((d.b, d.vn, 2), dtype=torch.float32, device=vertex.device)
    with torch.cuda.device(vertex.device):
        code = _lib.load().pv_ransac_motion_voting(ctypes.byref(d), out.data_ptr(),
                                                   torch.cuda.current_stream(vertex.device).cuda_stream)
    _lib.check(code, "ransac_motion_voting")
    return out


def ransac_voting_layer_v3_from_network(seg_pred, vertex_pred, round_hyp_num, inlier_thresh=0.99, confidence=0.99,
                                        max_iter=100, min_num=100, max_num=30000, *, _idxs=None, _keep=None,
                                        _diag=None, _seed=None, _workspace=None, out=None):
    """EvalWrapper (DEMO:46-55) fused: network outputs seg_pred [b,2,h,w] and
    vertex_pred [b,2vn,h,w] straight in -- the argmax and the permute/view are
    done inside the compaction kernel (no int64 mask, no strided copy)."""
    b, c, h, w = vertex_pred.shape
    vertex = vertex_pred.permute(0, 2, 3, 1).view(b, h, w, c // 2, 2)
    d = _desc(seg_pred, vertex, seg=True)
    return _v3(d, seg_pred, vertex, round_hyp_num, inlier_thresh, confidence, max_iter, min_num, max_num, _idxs,
               _keep, _diag, _seed, _workspace, out=out)


def _evd_common(mask, vertex, round_hyp_num, min_hyp_num, inlier_thresh, min_num, max_num, topk, _idxs, _keep,
                _seed, _workspace):
    d = _desc(mask, vertex)
    dev = vertex.device
    rounds = int(np.ceil(min_hyp_num / round_hyp_num))
    nh = rounds * round_hyp_num
    idxs = _aux(_idxs, torch.int32, dev, (d.b, nh, d.vn, 2), "_idxs")
    keep = _aux(_keep, torch.uint8, dev, (d.b, d.H, d.W), "_keep")
    prm = _params(round_hyp_num, inlier_thresh, 0.99, 100, min_num, max_num, _seed, idxs, keep,
                  min_hyp_num=min_hyp_num, topk=topk)
    L = _lib.load()
    nbytes = L.pv_v3_workspace_size(d.b, d.H, d.W, d.vn, nh)
    return d, prm, nbytes, (idxs, keep), _workspace or _default_ws


def estimate_voting_distribution_with_mean(mask, vertex, mean, round_hyp_num=256, min_hyp_num=4096, topk=128,
                                           inlier_thresh=0.99, min_num=20, max_num=30000, output_hyp=False, *,
                                           _idxs=None, _keep=None, _seed=None, _workspace=None):
    """RV:333-406 -> (mean, cov [b,vn,2,2]).  ``_idxs`` is [b, rounds*round_hyp_num, vn, 2]."""
    d, prm, nbytes, keepalive, work = _evd_common(mask, vertex, round_hyp_num, min_hyp_num, inlier_thresh, min_num,
                                                  max_num, topk, _idxs, _keep, _seed, _workspace)
    dev = vertex.device
    mean_c = mean.to(device=dev, dtype=torch.float32).contiguous()
    if tuple(mean_c.shape) != (d.b, d.vn, 2):
        raise RuntimeError("mean must be [b,vn,2]")
    cov = torch.empty((d.b, d.vn, 2, 2), dtype=torch.float32, device=dev)
    ws = work.get(dev, nbytes)
    with torch.cuda.device(dev):
        try:
            code = _lib.load().pv_estimate_voting_distribution_with_mean(
                ctypes.byref(d), ctypes.byref(prm), mean_c.data_ptr(), cov.data_ptr(), ws.data_ptr(), nbytes,
                torch.cuda.current_stream(dev).cuda_stream)
        finally:
            work.done(dev)
    _lib.check(code, "estimate_voting_distribution_with_mean")
    return mean, cov


def estimate_voting_distribution(mask, vertex, round_hyp_num=256, min_hyp_num=4096, topk=128, inlier_thresh=0.99,
                                 min_num=5, max_num=30000, *, _idxs=None, _keep=None, _seed=None, _workspace=None):
    """RV:263-331 -> (mean [b,vn,2], cov [b,vn,2,2]); topk ties lowest index first."""
    d, prm, nbytes, keepalive, work = _evd_common(mask, vertex, round_hyp_num, min_hyp_num, inlier_thresh, min_num,
                                                  max_num, topk, _idxs, _keep, _seed, _workspace)
    dev = vertex.device
    mean = torch.empty((d.b, d.vn, 2), dtype=torch.float32, device=dev)
    cov = torch.empty((d.b, d.vn, 2, 2), dtype=torch.float32, device=dev)
    ws = work.get(dev, nbytes)
    with torch.cuda.device(dev):
        try:
            code = _lib.load().pv_estimate_voting_distribution(
                ctypes.byref(d), ctypes.byref(prm), mean.data_ptr(), cov.data_ptr(), ws.data_ptr(), nbytes,
                torch.cuda.current_stream(dev).cuda_stream)
        finally:
            work.done(dev)
    _lib.check(code, "estimate_voting_distribution")
    return mean, cov


def b_inv(b_mat: torch.Tensor) -> torch.Tensor:
    """RV:503-518 with the semantics of the pinned torch (gesv present):
    batched inverse, or the identity for the WHOLE batch when any matrix is
    singular (the reference's bare ``except``)."""
    eye = b_mat.new_ones(b_mat.size(-1)).diag().expand_as(b_mat)
    try:
        return torch.linalg.solve(b_mat, eye)
    except RuntimeError:       # torch.linalg.LinAlgError subclasses RuntimeError
        return eye
