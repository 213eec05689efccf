"""Drop-in for the reference's compiled module ``ransac_voting``.

Same four functions, same positional signatures, same argument meaning as
``lib/ransac_voting_gpu_layer/src/ransac_voting.cpp:102-107`` (BND), so
``import pvnet_amd.ransac_voting as ransac_voting`` replaces
``import lib.ransac_voting_gpu_layer.ransac_voting as ransac_voting``
(ransac_voting_gpu.py:2).  Each call goes through the C ABI of libpvvote.so on
torch's current stream of the tensors' device.

Error behaviour follows BND:7-9 (``CHECK_INPUT``): a non-device or
non-contiguous tensor raises ``RuntimeError``.  Shapes are checked too (the
reference's C ``assert``s, KU:61-65 and KU:141-148, are compiled out under
NDEBUG; here they always raise).  A failing launch raises instead of calling
``exit()`` (cuda_common.h:19-26).
"""
from __future__ import annotations

import torch

from . import _lib


def _check_input(x: torch.Tensor, name: str):
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _check_dtype(x, dt, name):
    if x.dtype != dt:
        raise RuntimeError(f"{name} must be {dt}, got {x.dtype}")


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _common(direct, coords):
    _check_input(direct, "direct")
    _check_input(coords, "coords")
    _check_dtype(direct, torch.float32, "direct")
    _check_dtype(coords, torch.float32, "coords")
    if direct.dim() != 3 or direct.shape[2] != 2:
        raise RuntimeError("direct must be [tn,vn,2]")
    tn, vn = direct.shape[0], direct.shape[1]
    if coords.shape != (tn, 2):
        raise RuntimeError("coords must be [tn,2]")
    if coords.device != direct.device:
        raise RuntimeError("direct and coords must be on the same device")
    return tn, vn


def generate_hypothesis(direct: torch.Tensor, coords: torch.Tensor, idxs: torch.Tensor) -> torch.Tensor:
    """BND:20-31 / KU:51-86 -> f32 [hn,vn,2] on ``direct``'s device."""
    tn, vn = _common(direct, coords)
    _check_input(idxs, "idxs")
    _check_dtype(idxs, torch.int32, "idxs")
    if idxs.dim() != 3 or idxs.shape[1] != vn or idxs.shape[2] != 2:
        raise RuntimeError("idxs must be [hn,vn,2]")
    hn = idxs.shape[0]
    out = torch.empty((hn, vn, 2), dtype=torch.float32, device=direct.device)
    if hn:
        with torch.cuda.device(direct.device):
            _lib.check(_lib.load().pv_generate_hypothesis(direct.data_ptr(), coords.data_ptr(), idxs.data_ptr(),
                                                          out.data_ptr(), tn, vn, hn, _stream(direct.device)),
                       "generate_hypothesis")
    return out


def voting_for_hypothesis(direct, coords, hypo_pts, inliers, inlier_thresh) -> None:
    """BND:41-55 / KU:129-167: set ``inliers[h,v,t] = 1`` where pixel t votes
    for hypothesis (h,v); other bytes are left as they are (KU:124-125)."""
    _voting(direct, coords, hypo_pts, inliers, inlier_thresh, _lib.PV_VOTE_OR)


def voting_for_hypothesis_dense(direct, coords, hypo_pts, inliers, inlier_thresh) -> None:
    """Same decisions, but every byte of ``inliers`` is overwritten with 0/1.
    Identical to :func:`voting_for_hypothesis` on the zero tensors every
    reference call site passes (RV:563, RV:588, ...); used by the benchmark."""
    _voting(direct, coords, hypo_pts, inliers, inlier_thresh, _lib.PV_VOTE_DENSE)


def _voting(direct, coords, hypo_pts, inliers, thr, mode):
    tn, vn = _common(direct, coords)
    _check_input(hypo_pts, "hypo_pts")
    _check_input(inliers, "inliers")
    _check_dtype(hypo_pts, torch.float32, "hypo_pts")
    if inliers.dtype not in (torch.uint8, torch.bool):
        raise RuntimeError("inliers must be uint8")
    if hypo_pts.dim() != 3 or hypo_pts.shape[1] != vn or hypo_pts.shape[2] != 2:
        raise RuntimeError("hypo_pts must be [hn,vn,2]")
    hn = hypo_pts.shape[0]
    if tuple(inliers.shape) != (hn, vn, tn):
        raise RuntimeError("inliers must be [hn,vn,tn]")
    if tn == 0 or hn == 0:
        return
    L = _lib.load()
    with torch.cuda.device(direct.device):
        _lib.check(L.pv_voting_for_hypothesis(direct.data_ptr(), coords.data_ptr(), hypo_pts.data_ptr(),
                                              inliers.data_ptr(), tn, vn, hn, float(thr), mode,
                                              _stream(direct.device)), "voting_for_hypothesis")


def generate_hypothesis_vanishing_point(direct, coords, idxs) -> torch.Tensor:
    """BND:64-75 / KU:231-266 -> f32 [hn,vn,3]."""
    tn, vn = _common(direct, coords)
    _check_input(idxs, "idxs")
    _check_dtype(idxs, torch.int32, "idxs")
    if idxs.dim() != 3 or idxs.shape[1] != vn or idxs.shape[2] != 2:
        raise RuntimeError("idxs must be [hn,vn,2]")
    hn = idxs.shape[0]
    out = torch.empty((hn, vn, 3), dtype=torch.float32, device=direct.device)
    if hn:
        with torch.cuda.device(direct.device):
            _lib.check(_lib.load().pv_generate_hypothesis_vp(direct.data_ptr(), coords.data_ptr(), idxs.data_ptr(),
                                                             out.data_ptr(), tn, vn, hn, _stream(direct.device)),
                       "generate_hypothesis_vanishing_point")
    return out


def voting_for_hypothesis_vanishing_point(direct, coords, hypo_pts, inliers, inlier_thresh) -> None:
    """BND:85-99 / KU:313-351 (OR semantics)."""
    tn, vn = _common(direct, coords)
    _check_input(hypo_pts, "hypo_pts")
    _check_input(inliers, "inliers")
    if hypo_pts.dim() != 3 or hypo_pts.shape[1] != vn or hypo_pts.shape[2] != 3:
        raise RuntimeError("hypo_pts must be [hn,vn,3]")
    hn = hypo_pts.shape[0]
    if tuple(inliers.shape) != (hn, vn, tn):
        raise RuntimeError("inliers must be [hn,vn,tn]")
    with torch.cuda.device(direct.device):
        _lib.check(_lib.load().pv_voting_for_hypothesis_vp(direct.data_ptr(), coords.data_ptr(), hypo_pts.data_ptr(),
                                                           inliers.data_ptr(), tn, vn, hn, float(inlier_thresh),
                                                           _stream(direct.device)),
                   "voting_for_hypothesis_vanishing_point")


def vote_counts(direct, coords, hypo_pts, inlier_thresh) -> torch.Tensor:
    """Mask-free ``torch.sum(inliers, 2)`` of a fresh vote (RV:563-567): i32 [hn,vn]."""
    tn, vn = _common(direct, coords)
    _check_input(hypo_pts, "hypo_pts")
    hn = hypo_pts.shape[0]
    out = torch.empty((hn, vn), dtype=torch.int32, device=direct.device)
    with torch.cuda.device(direct.device):
        _lib.check(_lib.load().pv_vote_counts(direct.data_ptr(), coords.data_ptr(), hypo_pts.data_ptr(),
                                              out.data_ptr(), tn, vn, hn, float(inlier_thresh),
                                              _stream(direct.device)), "vote_counts")
    return out
