"""Load the golden fixtures and rebuild their inputs (no reference code needed)."""
from __future__ import annotations

import hashlib
import os

import numpy as np

from pvnet_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def cat_inputs(g):
    """LINEMOD 'cat' demo (tools/demo.py:74-103): int64 mask [1,h,w], vertex
    view [1,h,w,9,2] (of the network layout), network-layout vertex [1,18,h,w]."""
    mask = np.unpackbits(g["mask_bits"])[: 480 * 640].reshape(480, 640).astype(np.int32)
    field = synth.gt_vertex_field(mask, g["points_2d"])
    assert sha(field) == str(g["field_sha"]), "GT field generator drifted"
    vnet = synth.to_network_layout(field)
    vertex = np.ascontiguousarray(vnet.transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
    return mask.astype(np.int64)[None], vertex, vnet


def synth_inputs(g):
    f = synth.synthetic_field(int(g["seed"]))
    assert sha(f["seg"]) == str(g["seg_sha"]) and sha(f["vertex"]) == str(g["vertex_sha"]), "S(seed) drifted"
    mask = np.argmax(f["seg"], 1).astype(np.int64)
    vertex = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
    return mask, vertex, f


def ycb_inputs(g):
    """configs[4] frame of ycb21_cases: 21 keypoints projected from a known
    pose (YCB camera), int64 mask [1,h,w], vertex view [1,h,w,21,2], field."""
    p2d = g["points_2d"]
    f = synth.synthetic_field(int(g["seed"]), vn=21, keypoints=p2d,
                              center=(float(p2d[:, 0].mean()), float(p2d[:, 1].mean())))
    assert sha(f["seg"]) == str(g["seg_sha"]) and sha(f["vertex"]) == str(g["vertex_sha"]), "S(seed) drifted"
    mask = np.argmax(f["seg"], 1).astype(np.int64)
    vertex = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, 480, 640, 21, 2))
    return mask, vertex, f
