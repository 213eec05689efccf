"""Synthetic and known-answer inputs for the voting hot path.

* :func:`synthetic_field` is the generator S(seed) of SURVEY.md 8(d): a 480x640
  frame with a disk-shaped object (r = 97.5 px -> 29,861 foreground pixels,
  below ``max_num`` = 30000 so no downsampling RNG is involved), 9 keypoints,
  a unit direction field with N(0, 0.05 rad) angular noise and 20 % outliers,
  laid out the way the network emits it (``vertex_pred`` [1,2K,H,W] and
  ``seg_pred`` [1,2,H,W] whose argmax is the disk).
* :func:`gt_vertex_field` restates ``compute_vertex`` (tools/demo.py:58-71),
  and :func:`project` restates ``Projector.project`` (lib/utils/base_utils.py:
  252-256) with the LINEMOD intrinsics (base_utils.py:241-243): together with
  the LINEMOD 'cat' demo pose they give a field whose keypoints are known.
"""
from __future__ import annotations

import numpy as np

LINEMOD_K = np.array([[572.4114, 0., 325.2611],
                      [0., 573.57043, 242.04899],
                      [0., 0., 1.]])


def disk_mask(H=480, W=640, center=(320.0, 240.0), radius=97.5):
    yy, xx = np.mgrid[0:H, 0:W]
    return ((xx - center[0]) ** 2 + (yy - center[1]) ** 2) <= radius * radius


def synthetic_field(seed=1234, H=480, W=640, vn=9, radius=97.5, center=(320.0, 240.0),
                    noise=0.05, outlier=0.2, scale_jitter=False, mask=None, dtype=np.float32, keypoints=None):
    """S(seed): returns dict(seg [1,2,H,W], vertex [1,2vn,H,W], mask [H,W] bool,
    keypoints [vn,2] float64).  numpy ``default_rng(seed)`` only."""
    rng = np.random.default_rng(seed)
    m = disk_mask(H, W, center, radius) if mask is None else np.asarray(mask, bool)
    kps = rng.uniform([200.0, 120.0], [440.0, 360.0], size=(vn, 2))
    if keypoints is not None:      # e.g. projected model keypoints (the PnP tests)
        kps = np.asarray(keypoints, np.float64).reshape(vn, 2)
    rows, cols = np.nonzero(m)
    tn = rows.shape[0]
    ang = np.arctan2(kps[None, :, 1] - rows[:, None], kps[None, :, 0] - cols[:, None])  # [tn,vn]
    ang = ang + rng.normal(0.0, noise, size=ang.shape)
    out = rng.random(size=ang.shape) < outlier
    ang = np.where(out, rng.uniform(-np.pi, np.pi, size=ang.shape), ang)
    scale = rng.uniform(0.5, 1.5, size=ang.shape) if scale_jitter else 1.0
    vx, vy = np.cos(ang) * scale, np.sin(ang) * scale
    vertex = np.zeros((1, 2 * vn, H, W), dtype)
    vertex[0, 0::2][:, rows, cols] = vx.T.astype(dtype)
    vertex[0, 1::2][:, rows, cols] = vy.T.astype(dtype)
    seg = np.zeros((1, 2, H, W), dtype)
    seg[0, 1] = np.where(m, 1.0, -1.0).astype(dtype)
    return dict(seg=seg, vertex=vertex, mask=m, keypoints=kps, tn=tn)


def field_keypoints(seed=1234, vn=9):
    """The keypoints of S(seed) (synthetic_field's first draw) without
    building the field: lets a rank check the stream order of images it never
    held."""
    return np.random.default_rng(seed).uniform([200.0, 120.0], [440.0, 360.0], size=(vn, 2))


STREAM_KINDS = ("full", "split", "tiny", "large", "corner", "empty", "border", "small")


def stream_mask(kind, rng, H=480, W=640):
    """Foreground of one configs[3] (Occlusion-LINEMOD stream) frame, SURVEY.md
    8(d)4.  The stream mixes:

    * ``full``   the LINEMOD-cat-sized disk (r 97.5, 29,861 px);
    * ``split``  an occluded split disk: a disk cut in two by a vertical
                 occluder band (two pieces, the reference sees one mask);
    * ``tiny``   a mask below ``min_num`` (< 100 px): the zeros path, RV:537-540;
    * ``large``  a disk above ``max_num`` (> 30,000 px): Bernoulli
                 downsampling, RV:543-546;
    * ``corner`` a disk with one quadrant occluded;
    * ``empty``  no foreground at all;
    * ``border`` a disk clipped by the image border;
    * ``small``  a mask just above ``min_num`` (~100-200 px).

    Centres and sizes are drawn from ``rng`` (numpy Generator)."""
    yy, xx = np.mgrid[0:H, 0:W]

    def disk(cx, cy, r):
        return (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r

    cx, cy = rng.uniform(0.3 * W, 0.7 * W), rng.uniform(0.3 * H, 0.7 * H)
    if kind == "full":
        return disk(320.0, 240.0, 97.5)
    if kind == "split":
        r = rng.uniform(70, 100)
        band = rng.uniform(0.15, 0.35) * r
        off = rng.uniform(-0.3, 0.3) * r
        return disk(cx, cy, r) & ~(np.abs(xx - cx - off) < band)
    if kind == "tiny":
        return disk(cx, cy, rng.uniform(2.0, 5.0))
    if kind == "large":
        return disk(cx, cy, rng.uniform(105, 130))
    if kind == "corner":
        m = disk(cx, cy, rng.uniform(60, 95))
        return m & ~((xx > cx) & (yy < cy))
    if kind == "empty":
        return np.zeros((H, W), bool)
    if kind == "border":
        return disk(rng.uniform(-30, 40), rng.uniform(-30, H + 30), rng.uniform(80, 120))
    if kind == "small":
        return disk(cx, cy, rng.uniform(6.0, 7.5))
    raise ValueError(kind)


def stream_field(i, seed=9000, H=480, W=640, vn=9, **kw):
    """Image i of the configs[3] stream: kind ``STREAM_KINDS[i % 8]``
    (:func:`stream_mask`), field and keypoints as :func:`synthetic_field`
    with seed ``seed + i``.  Returns synthetic_field's dict plus ``kind``."""
    kind = STREAM_KINDS[i % len(STREAM_KINDS)]
    m = stream_mask(kind, np.random.default_rng(seed + 7919 * i), H, W)
    f = synthetic_field(seed + i, H=H, W=W, vn=vn, mask=m, **kw)
    f["kind"] = kind
    return f


def keep_mask(fg, max_num, rng):
    """A downsampling keep-mask for a foreground above ``max_num``: the
    reference's ``uniform_(0, 1) < max_num / fg`` (RV:543-546), drawn on the
    host so that a test can inject it into both sides."""
    fgn = int(np.count_nonzero(fg))
    if fgn <= max_num:
        return np.ones(fg.shape, np.uint8)
    return (rng.random(fg.shape, dtype=np.float32) < np.float32(np.float32(max_num) / np.float32(fgn))).astype(np.uint8)


def synthetic_batch(b, seed=1234, **kw):
    """b images S(seed), S(seed+1), ... stacked on dim 0."""
    fs = [synthetic_field(seed + i, **kw) for i in range(b)]
    return dict(seg=np.concatenate([f["seg"] for f in fs]), vertex=np.concatenate([f["vertex"] for f in fs]),
                mask=np.stack([f["mask"] for f in fs]), keypoints=np.stack([f["keypoints"] for f in fs]))


def project(pts_3d, RT, K=LINEMOD_K):
    """Projector.project (lib/utils/base_utils.py:252-256)."""
    p = np.matmul(pts_3d, RT[:, :3].T) + RT[:, 3:].T
    p = np.matmul(p, K.T)
    return p[:, :2] / p[:, 2:]


def gt_vertex_field(mask, points_2d):
    """compute_vertex (tools/demo.py:58-71): [h,w,2m] float32 unit vectors from
    each foreground pixel (mask == 1) to each keypoint, zero elsewhere."""
    mask = np.asarray(mask)
    m = points_2d.shape[0]
    h, w = mask.shape
    xy = np.argwhere(mask == 1)[:, [1, 0]]
    v = xy[:, None, :] * np.ones(shape=[1, m, 1])
    v = points_2d[None, :, :2] - v
    norm = np.linalg.norm(v, axis=2, keepdims=True)
    norm[norm < 1e-3] += 1e-3
    v = v / norm
    out = np.zeros([h, w, m, 2], np.float32)
    out[xy[:, 1], xy[:, 0]] = v
    return np.reshape(out, [h, w, m * 2])


def to_network_layout(vertex_hw2k):
    """[h,w,2K] -> vertex_pred layout [1,2K,h,w] (what the network emits)."""
    return np.ascontiguousarray(np.transpose(vertex_hw2k, (2, 0, 1))[None])
