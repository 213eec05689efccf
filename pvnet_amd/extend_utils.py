"""Uncertainty-weighted PnP on the device -- drop-in for the reference's
``lib.utils.extend_utils.extend_utils.uncertainty_pnp`` / ``uncertainty_pnp_v2``
(extend_utils.py:63-166) and for the covariance -> weight step of
``Evaluator.evaluate_uncertainty`` (lib/utils/evaluation_utils.py:161-190).

The reference runs, per image and on the host, ``cv2.solvePnP(SOLVEPNP_P3P)``
for an initial pose and then Ceres (src/uncertainty_pnp.cpp) through cffi.
Here the whole stage is one batched HIP kernel (``pv_uncertainty_pnp``: one
wave per image, fp64) behind the same Python signatures:

* ``uncertainty_pnp(points_2d, weights_2d, points_3d, camera_matrix)`` and
  ``uncertainty_pnp_v2(points_2d, covars, points_3d, camera_matrix)`` take
  and return numpy arrays like the reference (Rt [3, 4] float64) and run on
  the current ROCm device;
* ``uncertainty_pnp_batch`` is the batched device form (torch tensors in,
  Rt [b, 3, 4] float64 out, on the inputs' device and current stream), fed
  directly by ``estimate_voting_distribution_with_mean``'s (mean, cov).

No CPU fallback: without libpvvote.so or a ROCm device the calls raise.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_MODES = {"weights": _lib.PV_PNP_WEIGHTS, "cov": _lib.PV_PNP_COV, "cov_v2": _lib.PV_PNP_COV_V2}


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("uncertainty_pnp runs on the ROCm device (no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def uncertainty_pnp_batch(points_2d: torch.Tensor, wgt: torch.Tensor, points_3d, camera_matrix, mode: str = "cov",
                          init_rt: torch.Tensor | None = None, diag: dict | None = None) -> torch.Tensor:
    """Batched uncertainty PnP on the device.

    points_2d  [b, pn, 2] the voted keypoints (e.g. ransac_voting_layer_v3's output); float64
               points are used at full precision (the reference's single-image path passes
               float64, extend_utils.py:80), anything else as float32
    wgt        mode "cov" / "cov_v2": f32 [b, pn, 2, 2] covariances (estimate_voting_distribution*);
               mode "weights": f64 [b, pn, 3] (wxx, wxy, wyy)
    points_3d  f64 [pn, 3] shared, or [b, pn, 3]
    camera_matrix f64 [3, 3] shared, or [b, 3, 3]
    init_rt    optional f64 [b, 6]: skip the P3P initialisation and refine from these poses
               (src/uncertainty_pnp.cpp:58-92; mode "weights" only); the result is then [b, 6]
    Returns Rt f64 [b, 3, 4] (or the refined [b, 6] poses with init_rt).
    """
    if mode not in _MODES:
        raise ValueError(f"mode must be one of {sorted(_MODES)}")
    dev = points_2d.device
    if dev.type != "cuda":
        raise RuntimeError("points_2d must be a device tensor")
    b, pn = int(points_2d.shape[0]), int(points_2d.shape[1])
    if points_2d.dim() != 3 or points_2d.shape[2] != 2:
        raise RuntimeError("points_2d must be [b, pn, 2]")
    if not 4 <= pn <= 64:
        raise RuntimeError("uncertainty_pnp needs 4 <= pn <= 64 points per image")
    p2 = points_2d.contiguous() if points_2d.dtype == torch.float64 else points_2d.to(torch.float32).contiguous()
    if mode == "weights":
        w = wgt.to(device=dev, dtype=torch.float64).contiguous()
        if tuple(w.shape) != (b, pn, 3):
            raise RuntimeError("weights must be [b, pn, 3]")
    else:
        w = wgt.to(device=dev, dtype=torch.float32).contiguous()
        if tuple(w.shape) != (b, pn, 2, 2):
            raise RuntimeError("covariances must be [b, pn, 2, 2]")
    p3 = torch.as_tensor(points_3d, dtype=torch.float64).to(dev).contiguous()
    K = torch.as_tensor(camera_matrix, dtype=torch.float64).to(dev).contiguous()
    if p3.dim() == 2:
        if tuple(p3.shape) != (pn, 3):
            raise RuntimeError("points_3d must be [pn, 3] or [b, pn, 3]")
        p3s = 0
    elif tuple(p3.shape) == (b, pn, 3):
        p3s = pn * 3
    else:
        raise RuntimeError("points_3d must be [pn, 3] or [b, pn, 3]")
    if K.dim() == 2:
        if tuple(K.shape) != (3, 3):
            raise RuntimeError("camera_matrix must be [3, 3] or [b, 3, 3]")
        ks = 0
    elif tuple(K.shape) == (b, 3, 3):
        ks = 9
    else:
        raise RuntimeError("camera_matrix must be [3, 3] or [b, 3, 3]")
    f64 = p2.dtype == torch.float64
    bt = _lib.PnpBatch(b, pn, _MODES[mode], None if f64 else p2.data_ptr(), w.data_ptr(), p3.data_ptr(), K.data_ptr(),
                       p3s, ks, p2.data_ptr() if f64 else None)
    dg = _lib.PnpDiag()
    keep = []
    if diag is not None:
        d = dict(init_rt=torch.zeros((b, 6), dtype=torch.float64, device=dev),
                 p3p_ok=torch.zeros(b, dtype=torch.int32, device=dev),
                 iterations=torch.zeros(b, dtype=torch.int32, device=dev),
                 status=torch.zeros(b, dtype=torch.int32, device=dev),
                 cost=torch.zeros(b, dtype=torch.float64, device=dev))
        dg = _lib.PnpDiag(*(d[k].data_ptr() for k in ("init_rt", "p3p_ok", "iterations", "status", "cost")))
        keep.append(d)
    L = _lib.load()
    stream = torch.cuda.current_stream(dev).cuda_stream
    with torch.cuda.device(dev):
        if init_rt is not None:
            if mode != "weights":
                raise RuntimeError("init_rt needs mode='weights' (the reference C entry point takes weights)")
            x0 = init_rt.to(device=dev, dtype=torch.float64).contiguous()
            if tuple(x0.shape) != (b, 6):
                raise RuntimeError("init_rt must be [b, 6]")
            out = torch.empty((b, 6), dtype=torch.float64, device=dev)
            _lib.check(L.pv_uncertainty_pnp_refine(ctypes.byref(bt), x0.data_ptr(), out.data_ptr(), ctypes.byref(dg),
                                                   stream), "pv_uncertainty_pnp_refine")
        else:
            out = torch.empty((b, 3, 4), dtype=torch.float64, device=dev)
            _lib.check(L.pv_uncertainty_pnp(ctypes.byref(bt), out.data_ptr(), ctypes.byref(dg), stream),
                       "pv_uncertainty_pnp")
    if diag is not None:
        diag.update(keep[0])
    return out


def _single(points_2d, wgt, points_3d, camera_matrix, mode):
    pn = np.asarray(points_2d).shape[0]
    assert np.asarray(points_3d).shape[0] == pn and pn >= 4          # EU:72
    dev = _device()
    p2 = torch.from_numpy(np.ascontiguousarray(points_2d, np.float64)).to(dev)[None]   # EU:80
    w = np.ascontiguousarray(wgt, np.float64 if mode == "weights" else np.float32)
    w = torch.from_numpy(w).to(dev)[None]
    Rt = uncertainty_pnp_batch(p2, w, np.asarray(points_3d, np.float64), np.asarray(camera_matrix, np.float64), mode)
    return Rt[0].cpu().numpy()


def uncertainty_pnp(points_2d, weights_2d, points_3d, camera_matrix):
    """EU:63-114: points_2d [pn, 2], weights_2d [pn, 3] (wxx, wxy, wyy),
    points_3d [pn, 3], camera_matrix [3, 3] -> Rt [3, 4] float64."""
    return _single(points_2d, weights_2d, points_3d, camera_matrix, "weights")


def uncertainty_pnp_v2(points_2d, covars, points_3d, camera_matrix, type="single"):   # noqa: A002 (reference name)
    """EU:116-166: covars [pn, 2, 2] -> isotropic weights 1 / max eigenvalue -> Rt [3, 4]."""
    return _single(points_2d, covars, points_3d, camera_matrix, "cov_v2")


def pose_from_voting(mean: torch.Tensor, cov: torch.Tensor, points_3d, camera_matrix) -> torch.Tensor:
    """Evaluator.evaluate_uncertainty's pose step (evaluation_utils.py:161-187)
    for a batch: keypoints [b, vn, 2] and covariances [b, vn, 2, 2] from
    estimate_voting_distribution_with_mean -> Rt [b, 3, 4] (weights
    inv(sqrtm(cov)), zero for cov[0,0] < 1e-6 or NaN)."""
    return uncertainty_pnp_batch(mean, cov, points_3d, camera_matrix, "cov")
