"""ctypes binding of libpvvote.so (include/pvvote.h).

The product path has no CPU fallback: if the library is missing or the
tensors are not on a ROCm device, calls raise.  Build the library with
``python -m pvnet_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PVVOTE_LIB", os.path.join(HERE, "libpvvote.so"))

PV_MASK_I64, PV_MASK_U8, PV_MASK_I32, PV_MASK_SEG_F32, PV_MASK_SEG_F16 = 0, 1, 2, 3, 4
PV_VERTEX_F32, PV_VERTEX_F16 = 0, 1
PV_VOTE_OR, PV_VOTE_DENSE = 0, 1
PV_PNP_WEIGHTS, PV_PNP_COV, PV_PNP_COV_V2 = 0, 1, 2
PV_ACT_NONE, PV_ACT_RELU, PV_ACT_LEAKY = 0, 1, 2
PNP_STOP = {1: "gradient", 2: "parameter", 3: "function", 4: "max_iterations", 5: "radius", 6: "p3p_only"}

c_i32, c_i64, c_u64, c_f32, c_size, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float,
                                            ctypes.c_size_t, ctypes.c_void_p)


class ImageDesc(ctypes.Structure):
    _fields_ = [("mask", c_vp), ("mask_kind", c_i32), ("mask_strides", c_i64 * 4),
                ("vertex", c_vp), ("vertex_kind", c_i32), ("vertex_strides", c_i64 * 5),
                ("b", c_i32), ("H", c_i32), ("W", c_i32), ("vn", c_i32)]


class VoteParams(ctypes.Structure):
    _fields_ = [("round_hyp_num", c_i32), ("inlier_thresh", c_f32), ("confidence", c_f32),
                ("max_iter", c_i32), ("min_num", c_i32), ("max_num", c_i32), ("seed", c_u64),
                ("idxs", c_vp), ("keep", c_vp), ("min_hyp_num", c_i32), ("topk", c_i32)]


class V3Diag(ctypes.Structure):
    _fields_ = [("hyp", c_vp), ("counts", c_vp), ("win_idx", c_vp), ("win_ratio", c_vp), ("tn", c_vp),
                ("iters", c_vp), ("ata", c_vp), ("atb", c_vp), ("ev_vote_begin", c_vp), ("ev_vote_end", c_vp),
                ("ev_compact_end", c_vp)]


class PnpBatch(ctypes.Structure):
    _fields_ = [("b", c_i32), ("pn", c_i32), ("mode", c_i32), ("pts2d", c_vp), ("wgt", c_vp), ("pts3d", c_vp),
                ("K", c_vp), ("pts3d_stride", c_i64), ("K_stride", c_i64), ("pts2d64", c_vp)]


class PnpDiag(ctypes.Structure):
    _fields_ = [("init_rt", c_vp), ("p3p_ok", c_vp), ("iterations", c_vp), ("status", c_vp), ("cost", c_vp)]


# (name, restype, argtypes) -- one entry per function declared in include/pvvote.h
SIGNATURES = [
    ("pv_version", ctypes.c_char_p, []),
    ("pv_build_config", ctypes.c_char_p, []),
    ("pv_error_string", ctypes.c_char_p, [ctypes.c_int]),
    ("pv_device_arch", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    ("pv_stream_create", ctypes.c_int, [c_i32, ctypes.POINTER(c_vp)]),
    ("pv_stream_destroy", ctypes.c_int, [c_vp]),
    ("pv_stream_capture_id", ctypes.c_int, [c_vp, ctypes.POINTER(c_u64)]),
    ("pv_generate_hypothesis", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp]),
    ("pv_voting_for_hypothesis", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_i32, c_vp]),
    ("pv_generate_hypothesis_vp", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp]),
    ("pv_voting_for_hypothesis_vp", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_vote_counts", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_v3_workspace_size", c_size, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    ("pv_v3_kernel_launches", ctypes.c_int, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    ("pv_ransac_voting_v3", ctypes.c_int,
     [ctypes.POINTER(ImageDesc), ctypes.POINTER(VoteParams), c_vp, c_vp, c_size, ctypes.POINTER(V3Diag), c_vp]),
    ("pv_ransac_voting_v5", ctypes.c_int,
     [ctypes.POINTER(ImageDesc), ctypes.POINTER(VoteParams), c_f32, c_vp, c_vp, c_vp, c_size, ctypes.POINTER(V3Diag),
      c_vp]),
    ("pv_ransac_motion_voting", ctypes.c_int, [ctypes.POINTER(ImageDesc), c_vp, c_vp]),
    ("pv_estimate_voting_distribution_with_mean", ctypes.c_int,
     [ctypes.POINTER(ImageDesc), ctypes.POINTER(VoteParams), c_vp, c_vp, c_vp, c_size, c_vp]),
    ("pv_estimate_voting_distribution_with_mean_diag", ctypes.c_int,
     [ctypes.POINTER(ImageDesc), ctypes.POINTER(VoteParams), c_vp, c_vp, c_vp, c_size, ctypes.POINTER(V3Diag), c_vp]),
    ("pv_estimate_voting_distribution", ctypes.c_int,
     [ctypes.POINTER(ImageDesc), ctypes.POINTER(VoteParams), c_vp, c_vp, c_vp, c_size, c_vp]),
    ("pv_uncertainty_pnp", ctypes.c_int, [ctypes.POINTER(PnpBatch), c_vp, ctypes.POINTER(PnpDiag), c_vp]),
    ("pv_uncertainty_pnp_refine", ctypes.c_int,
     [ctypes.POINTER(PnpBatch), c_vp, c_vp, ctypes.POINTER(PnpDiag), c_vp]),
    ("pv_conv_epilogue_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_conv_epilogue_f32", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_head_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_vp]),
    ("pv_head_f32", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_vp]),
    ("pv_relu_maxpool_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    ("pv_relu_maxpool_f32", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    ("pv_conv3x3_f16", ctypes.c_int,
     [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_conv3x3_ex_f16", ctypes.c_int,
     [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32,
      c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp, c_i64, c_vp]),
    ("pv_conv3x3_workspace_bytes", c_i64, [c_i64, c_i32, c_i32]),
    ("pv_conv3x3_workspace_counter_bytes", c_i64, [c_i64, c_i32, c_i32]),
    ("pv_decoder_conv2s_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_decoder_conv4s_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_stem_conv_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp]),
    ("pv_stem_pool_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp]),
    ("pv_conv64_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    ("pv_decoder_tail_f16", ctypes.c_int,
     [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_decoder_tail_split_f16", ctypes.c_int,
     [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp]),
    ("pv_upsample2x_cat_f16", ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp]),
    ("pv_upsample2x_cat_f32", ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp]),
]

_lib = None
_lock = threading.Lock()


def load():
    """Load libpvvote.so once (raises if it is absent: no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libpvvote.so not found at {LIB_PATH}; build it with `python -m pvnet_amd.build`")
            L = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


class PVError(RuntimeError):
    pass


def check(code: int, what: str):
    if code != 0:
        msg = load().pv_error_string(code).decode()
        raise PVError(f"{what} failed: {msg} (code {code})")
