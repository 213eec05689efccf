"""Generate the golden vectors under tests/golden/ from the REFERENCE's own
Python voting layer (container-only; /root/reference does not exist on the GPU
box and nothing at test time imports it).

How the reference runs here:
  * ``lib/ransac_voting_gpu_layer/ransac_voting_gpu.py`` (RV) is executed from
    /root/reference unchanged.  Its CUDA extension cannot be built, so the
    module name it imports (RV:2) is bound to ``TorchKernels`` below: a
    torch-CPU restatement of ransac_voting_kernel.cu written independently of
    oracle/pvvote_oracle.c (elementwise fp32 ops, no contraction, double
    compares for the 1e-6 guards, correctly rounded sqrt/div via numpy).  Two restatements must then agree bit for
    bit in tests/test_oracle_golden.py.
  * ``Tensor.masked_select`` accepts the uint8 mask RV:550 passes (torch>=1.2
    requires bool); ``torch.gesv`` (gone from torch 2.x) is provided through
    ``torch.linalg.solve``, raising on a singular matrix like gesv did, so
    RV:514-517's identity fallback keeps its meaning.
  * The stub records every call (the idxs the reference drew, the hypotheses,
    the per-(h,v) inlier counts, the compacted coords) so the fixtures hold
    the reference's own intermediate values, not just its final output.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import hashlib
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("PVNET_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from pvnet_amd import synth  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _sqrt(x):
    """Correctly rounded fp32 sqrt.  torch-CPU's vectorised sqrt is not
    (1 ulp off on ~0.6 % of inputs here: AVX512 build), the CUDA kernel's
    sqrt is (nvcc -prec-sqrt=true default), numpy's sqrtps is."""
    return torch.from_numpy(np.sqrt(x.numpy()))


def _div(a, b):
    return torch.from_numpy(np.divide(a.numpy(), b.numpy()))


class TorchKernels:
    """Stand-in for the ``ransac_voting`` extension (BND:102-107)."""

    def __init__(self):
        self.calls = []
        self.forced = []          # queue of idxs arrays to impose on the next generate calls

    # KU:11-86
    def generate_hypothesis(self, direct, coords, idxs):
        if self.forced:
            idxs.copy_(torch.from_numpy(self.forced.pop(0)))
        t0, t1 = idxs[..., 0].long(), idxs[..., 1].long()
        v = torch.arange(direct.shape[1])[None]
        nx0, ny0 = direct[t0, v, 1], -direct[t0, v, 0]
        nx1, ny1 = direct[t1, v, 1], -direct[t1, v, 0]
        cx0, cy0 = coords[t0, 0], coords[t0, 1]
        cx1, cy1 = coords[t1, 0], coords[t1, 1]
        d0 = nx1 * ny0 - nx0 * ny1
        d1 = ny1 * nx0 - ny0 * nx1
        skip = (d0.abs().double() < 1e-6) | (d1.abs().double() < 1e-6)
        p0 = nx0 * cx0 + ny0 * cy0
        p1 = nx1 * cx1 + ny1 * cy1
        y = _div(nx1 * p0 - nx0 * p1, d0)
        x = _div(ny1 * p0 - ny0 * p1, d1)
        out = torch.zeros(idxs.shape[0], direct.shape[1], 2, dtype=torch.float32)
        out[..., 0] = torch.where(skip, torch.zeros_like(x), x)
        out[..., 1] = torch.where(skip, torch.zeros_like(y), y)
        self.calls.append(dict(kind="gen", idxs=idxs.clone().numpy(), hyp=out.clone().numpy(),
                               coords=coords.clone().numpy(), tn=int(direct.shape[0])))
        return out

    # KU:88-167
    def voting_for_hypothesis(self, direct, coords, hypo, inliers, thr):
        nx = direct[:, :, 0].t()[None]          # [1,vn,tn]
        ny = direct[:, :, 1].t()[None]
        cx = coords[:, 0][None, None]
        cy = coords[:, 1][None, None]
        norm1 = _sqrt(nx * nx + ny * ny)
        hn = hypo.shape[0]
        for h0 in range(0, hn, 16):
            hx = hypo[h0:h0 + 16, :, 0][..., None]
            hy = hypo[h0:h0 + 16, :, 1][..., None]
            dx = hx - cx
            dy = hy - cy
            norm2 = _sqrt(dx * dx + dy * dy)
            ok = ~((norm1.double() < 1e-6) | (norm2.double() < 1e-6))
            ad = _div(dx * nx + dy * ny, norm1 * norm2)
            hit = ok & (ad > thr)
            inliers[h0:h0 + 16][hit] = 1
        self.calls.append(dict(kind="vote", hyp=hypo.clone().numpy(),
                               counts=inliers.long().sum(2).numpy(), tn=int(direct.shape[0])))

    # KU:170-266
    def generate_hypothesis_vanishing_point(self, direct, coords, idxs):
        t0, t1 = idxs[..., 0].long(), idxs[..., 1].long()
        v = torch.arange(direct.shape[1])[None]
        dx0, dy0, dx1, dy1 = direct[t0, v, 0], direct[t0, v, 1], direct[t1, v, 0], direct[t1, v, 1]
        cx0, cy0, cx1, cy1 = coords[t0, 0], coords[t0, 1], coords[t1, 0], coords[t1, 1]
        lx0, ly0, lz0 = dy0, -dx0, cy0 * dx0 - cx0 * dy0
        lx1, ly1, lz1 = dy1, -dx1, cy1 * dx1 - cx1 * dy1
        x = ly0 * lz1 - lz0 * ly1
        y = lz0 * lx1 - lx0 * lz1
        z = lx0 * ly1 - ly0 * lx1
        vx0, vx1 = dx0 * (x - z * cx0), dx1 * (x - z * cx1)
        vy0, vy1 = dy0 * (y - z * cy0), dy1 * (y - z * cy1)
        flip = (vx0 < 0) & (vx1 < 0) & (vy0 < 0) & (vy1 < 0)
        x, y, z = torch.where(flip, -x, x), torch.where(flip, -y, y), torch.where(flip, -z, z)
        bad = (vx0 * vx1 < 0) | (vy0 * vy1 < 0)
        zero = torch.zeros_like(x)
        return torch.stack([torch.where(bad, zero, x), torch.where(bad, zero, y), torch.where(bad, zero, z)], -1)

    # KU:268-351
    def voting_for_hypothesis_vanishing_point(self, direct, coords, hypo, inliers, thr):
        ddx = direct[:, :, 0].t()[None]
        ddy = direct[:, :, 1].t()[None]
        cx = coords[:, 0][None, None]
        cy = coords[:, 1][None, None]
        hx, hy, hz = hypo[..., 0][..., None], hypo[..., 1][..., None], hypo[..., 2][..., None]
        fx = hx - cx * hz
        fy = hy - cy * hz
        n1 = _sqrt(ddx * ddx + ddy * ddy)
        n2 = _sqrt(fx * fx + fy * fy)
        ok = ~((n1.double() < 1e-6) | (n2.double() < 1e-6))
        ad = _div(ddx * fx + ddy * fy, n1 * n2)
        ok = ok & ~((fx * ddx < 0) | (fy * ddy < 0)) & (ad.abs() > thr)
        inliers[ok] = 1


def load_reference(stub: TorchKernels):
    lib = types.ModuleType("lib")
    lib.__path__ = []
    sub = types.ModuleType("lib.ransac_voting_gpu_layer")
    sub.__path__ = []
    lib.ransac_voting_gpu_layer = sub
    sub.ransac_voting = stub
    sys.modules.update({"lib": lib, "lib.ransac_voting_gpu_layer": sub,
                        "lib.ransac_voting_gpu_layer.ransac_voting": stub})
    path = os.path.join(REF, "lib", "ransac_voting_gpu_layer", "ransac_voting_gpu.py")
    spec = importlib.util.spec_from_file_location("reference_rv", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def install_shims():
    orig = torch.Tensor.masked_select

    def masked_select(self, m):
        return orig(self, m.bool() if m.dtype == torch.uint8 else m)

    torch.Tensor.masked_select = masked_select

    def gesv(B, A):
        return torch.linalg.solve(A, B), None     # raises LinAlgError on singular A, as gesv did

    torch.gesv = gesv


def demo_cat():
    from PIL import Image
    d = os.path.join(REF, "data", "demo")
    mask = np.array(Image.open(os.path.join(d, "cat_mask.png"))).astype(np.int32)[..., 0]
    mask[mask != 0] = 1
    pts3d = np.loadtxt(os.path.join(d, "cat_points_3d.txt"))
    pose = np.load(os.path.join(d, "cat_pose.npy"))
    p2d = synth.project(pts3d, pose)
    return mask, pts3d, pose, p2d


def vote_calls(stub, kind):
    return [c for c in stub.calls if c["kind"] == kind]


def run_v3(RV, stub, mask, vertex, hn, **kw):
    stub.calls.clear()
    out = RV.ransac_voting_layer_v3(torch.from_numpy(mask), torch.from_numpy(vertex), hn, **kw)
    return out.numpy()


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path), "bytes")


def per_image_records(stub):
    """Group stub calls per image for v3: first gen+vote of each image, then the
    refine vote (hn=1).  Returns lists idxs, hyps, counts, refine_counts, coords."""
    idxs, hyps, counts, refc, coords = [], [], [], [], []
    i = 0
    calls = stub.calls
    while i < len(calls):
        c = calls[i]
        if c["kind"] == "gen":
            idxs.append(c["idxs"]); hyps.append(c["hyp"]); coords.append(c["coords"])
            counts.append(calls[i + 1]["counts"])
            # skip repeated (identical) iterations
            j = i + 2
            while j < len(calls) and calls[j]["kind"] == "gen":
                j += 2
            refc.append(calls[j]["counts"][0])
            i = j + 1
        else:
            i += 1
    return idxs, hyps, counts, refc, coords


def main():
    install_shims()
    stub = TorchKernels()
    RV = load_reference(stub)

    # ---- G1: LINEMOD cat, ground-truth field (DEMO:74-103) ---------------
    mask, pts3d, pose, p2d = demo_cat()
    field = synth.gt_vertex_field(mask, p2d)                     # [h,w,18]
    vnet = synth.to_network_layout(field)                         # [1,18,h,w]
    vertex = torch.from_numpy(vnet).permute(0, 2, 3, 1).reshape(1, 480, 640, 9, 2).numpy()
    m64 = mask.astype(np.int64)[None]
    cat_in = dict(mask_bits=np.packbits(mask.astype(bool)), points_2d=p2d, pose=pose, points_3d=pts3d,
                  field_sha=sha(field))

    torch.manual_seed(0)
    kp = run_v3(RV, stub, m64, vertex, 512, inlier_thresh=0.99)                 # DEMO:55
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    iters = len(vote_calls(stub, "gen"))
    save("cat_v3_512", keypoints=kp, idxs=np.stack(idxs), hyp=np.stack(hyps), counts=np.stack(counts),
         refine_counts=np.stack(refc), iters=iters, err_vs_gt=np.abs(kp[0] - p2d).max(), **cat_in)
    print("cat v3 max err vs projection", np.abs(kp[0] - p2d).max(), "iters", iters)

    torch.manual_seed(1)
    mean = torch.from_numpy(kp)
    stub.calls.clear()
    m_, cov = RV.estimate_voting_distribution_with_mean(torch.from_numpy(m64), torch.from_numpy(vertex), mean)
    gens = vote_calls(stub, "gen")
    save("cat_evdm", mean=kp, cov=cov.numpy(), idxs=np.stack([g["idxs"] for g in gens])[None],
         counts=np.stack([c["counts"] for c in vote_calls(stub, "vote")])[None], **cat_in)

    torch.manual_seed(2)
    kp = run_v3(RV, stub, m64, vertex, 128, inlier_thresh=0.99, max_num=100)      # TRAIN:125
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    keep = np.zeros((480, 640), bool)
    keep[coords[0][:, 1].astype(int), coords[0][:, 0].astype(int)] = True
    save("cat_v3_128_maxnum100", keypoints=kp, idxs=np.stack(idxs), hyp=np.stack(hyps),
         counts=np.stack(counts), refine_counts=np.stack(refc), keep_bits=np.packbits(keep)[None], **cat_in)

    # ---- G2: synthetic S(1234) ------------------------------
    f = synth.synthetic_field(1234)
    seg = torch.from_numpy(f["seg"])
    vnet = torch.from_numpy(f["vertex"])
    m = torch.argmax(seg, 1)                                                      # DEMO:52
    vv = vnet.permute(0, 2, 3, 1).reshape(1, 480, 640, 9, 2)                       # DEMO:48-50
    syn_in = dict(seed=1234, seg_sha=sha(f["seg"]), vertex_sha=sha(f["vertex"]), mask_sha=sha(m.numpy()))
    for hn, seed in ((512, 3), (128, 4)):
        torch.manual_seed(seed)
        stub.calls.clear()
        kp = RV.ransac_voting_layer_v3(m, vv, hn, inlier_thresh=0.99).numpy()
        idxs, hyps, counts, refc, coords = per_image_records(stub)
        save(f"synth_v3_{hn}", keypoints=kp, idxs=np.stack(idxs), hyp=np.stack(hyps), counts=np.stack(counts),
             refine_counts=np.stack(refc), iters=len(vote_calls(stub, "gen")), **syn_in)
        if hn == 512:
            mean = torch.from_numpy(kp)
    torch.manual_seed(5)
    stub.calls.clear()
    _, cov = RV.estimate_voting_distribution_with_mean(m, vv, mean)
    gens = vote_calls(stub, "gen")
    save("synth_evdm", mean=mean.numpy(), cov=cov.numpy(), idxs=np.stack([g["idxs"] for g in gens])[None],
         counts=np.stack([c["counts"] for c in vote_calls(stub, "vote")])[None], **syn_in)
    for topk, seed in ((4096, 6), (128, 7)):
        torch.manual_seed(seed)
        stub.calls.clear()
        mu, cov = RV.estimate_voting_distribution(m, vv, topk=topk)
        gens = vote_calls(stub, "gen")
        save(f"synth_evd_top{topk}", mean=mu.numpy(), cov=cov.numpy(),
             idxs=np.stack([g["idxs"] for g in gens])[None], **syn_in)

    # ---- G3: edge cases on small frames -----------------------------------
    edge_cases(RV, stub)
    v5_cases(RV, stub, m64, vertex, cat_in)
    motion_cases(RV)
    vp_kernels(stub)


def small_field(seed, H=40, W=48, vn=3, radius=14.5, center=(24.0, 20.0), **kw):
    f = synth.synthetic_field(seed, H=H, W=W, vn=vn, radius=radius, center=center, **kw)
    vv = np.ascontiguousarray(f["vertex"][0].transpose(1, 2, 0).reshape(H, W, vn, 2))
    return f, vv


def edge_cases(RV, stub):
    H, W, vn = 40, 48, 3
    out = {}

    # (a) batch mixing: normal / too-few-foreground / int64 mask values 2,256,257
    fa, va = small_field(11)
    fb, vb = small_field(12, radius=4.0)                 # 49 px < min_num=100 -> zeros
    fc, vc = small_field(13)
    mc = fc["mask"].astype(np.int64)
    mc[mc == 1] = np.array([1, 2, 256, 257])[np.arange(int(mc.sum())) % 4]   # byte(): 256 -> 0
    masks = np.stack([fa["mask"].astype(np.int64), fb["mask"].astype(np.int64), mc])
    verts = np.stack([va, vb, vc])
    torch.manual_seed(10)
    kp = run_v3(RV, stub, masks, verts, 64)
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    out.update(a_mask=masks, a_vertex=verts, a_keypoints=kp, a_idxs=np.stack(idxs), a_hyp=np.stack(hyps),
               a_counts=np.stack(counts), a_refine_counts=np.stack(refc))
    torch.manual_seed(11)
    stub.calls.clear()
    mu = torch.from_numpy(kp)
    _, cov = RV.estimate_voting_distribution_with_mean(torch.from_numpy(masks), torch.from_numpy(verts), mu,
                                                       round_hyp_num=32, min_hyp_num=100)
    gens = vote_calls(stub, "gen")
    # images 0 and 2 voted (image 1 below min_num=20? no: 49 >= 20) -> 4 rounds each
    out.update(a_evdm_cov=cov.numpy(), a_evdm_idxs=np.stack([g["idxs"] for g in gens]))

    # (b) one keypoint with an all-zero field: no inliers -> singular ATA ->
    #     RV:514-517 identity for every keypoint; stop rule never met -> 101 iterations
    fz, vz = small_field(14)
    vz = vz.copy()
    vz[:, :, 1, :] = 0.0
    torch.manual_seed(12)
    kp = run_v3(RV, stub, fz["mask"].astype(np.int64)[None], vz[None], 32)
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    out.update(b_mask=fz["mask"].astype(np.int64)[None], b_vertex=vz[None], b_keypoints=kp, b_idxs=np.stack(idxs),
               b_hyp=np.stack(hyps), b_counts=np.stack(counts), b_refine_counts=np.stack(refc),
               b_iters=len(vote_calls(stub, "gen")))

    # (c) forced idxs: t0 == t1, parallel lines, a hypothesis exactly on a pixel
    #     centre (norm2 == 0), duplicate hypotheses (count ties -> first index)
    m = np.zeros((H, W), np.int64)
    m[5:35, 6:40] = 1
    rows, cols = np.nonzero(m)
    tn = rows.shape[0]
    rng = np.random.default_rng(15)
    vv = np.zeros((H, W, vn, 2), np.float32)
    ang = rng.uniform(-np.pi, np.pi, size=(tn, vn))
    vv[rows, cols, :, 0] = np.cos(ang)
    vv[rows, cols, :, 1] = np.sin(ang)
    lin = {(r, c): i for i, (r, c) in enumerate(zip(rows, cols))}
    # pixel A=(x=10,y=20) pointing +x (line y=20), pixel B=(x=30,y=8) pointing +y (line x=30):
    # they intersect exactly at pixel (30,20), which is in the mask.
    vv[20, 10, 0] = (1.0, 0.0)
    vv[8, 30, 0] = (0.0, 1.0)
    vv[12, 15, 0] = (0.0, 0.0)      # a zero-direction pixel (norm1 == 0)
    ia, ib = lin[(20, 10)], lin[(8, 30)]
    hn = 16
    forced = rng.integers(0, tn, size=(hn, vn, 2)).astype(np.int32)
    forced[0, 0] = (ia, ib)          # exact intersection on a pixel centre
    forced[1, 0] = (ia, ia)          # t0 == t1 -> degenerate -> (0,0)
    forced[2, 0] = (ib, ia)          # same point as h=0 -> tie, first index wins
    forced[3, 0] = (lin[(12, 15)], ia)   # zero direction -> degenerate
    forced[5] = forced[4]            # whole duplicate hypothesis row
    stub.forced = [forced]
    torch.manual_seed(13)
    kp = run_v3(RV, stub, m[None], vv[None], hn)
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    out.update(c_mask=m[None], c_vertex=vv[None], c_keypoints=kp, c_idxs=np.stack(idxs), c_hyp=np.stack(hyps),
               c_counts=np.stack(counts), c_refine_counts=np.stack(refc))

    # (d) downsampling: fg > max_num, keep-mask recovered from the compacted coords
    fd, vd = small_field(16)
    torch.manual_seed(14)
    kp = run_v3(RV, stub, fd["mask"].astype(np.int64)[None], vd[None], 32, max_num=300)
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    keep = np.zeros((H, W), bool)
    keep[coords[0][:, 1].astype(int), coords[0][:, 0].astype(int)] = True
    out.update(d_mask=fd["mask"].astype(np.int64)[None], d_vertex=vd[None], d_keypoints=kp, d_idxs=np.stack(idxs),
               d_hyp=np.stack(hyps), d_counts=np.stack(counts), d_refine_counts=np.stack(refc),
               d_keep=keep[None])

    # (e) scale-jittered field (|direction| in [0.5,1.5]) and thr 0.999 (RV v5's second threshold)
    fe, ve = small_field(17, scale_jitter=True)
    torch.manual_seed(15)
    kp = run_v3(RV, stub, fe["mask"].astype(np.int64)[None], ve[None], 48, inlier_thresh=0.999)
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    out.update(e_mask=fe["mask"].astype(np.int64)[None], e_vertex=ve[None], e_keypoints=kp, e_idxs=np.stack(idxs),
               e_hyp=np.stack(hyps), e_counts=np.stack(counts), e_refine_counts=np.stack(refc))
    save("edge_cases", **out)


def v5_records(stub):
    """Per image of ransac_voting_layer_v5 (RV:769-864): the first gen+vote,
    then the refine vote (hn=1) and the confidence vote (hn=1, thr 0.999)."""
    idxs, hyps, counts, refc, confc, coords = [], [], [], [], [], []
    calls, i = stub.calls, 0
    while i < len(calls):
        c = calls[i]
        if c["kind"] == "gen":
            idxs.append(c["idxs"]); hyps.append(c["hyp"]); coords.append(c["coords"])
            counts.append(calls[i + 1]["counts"])
            j = i + 2
            while j < len(calls) and calls[j]["kind"] == "gen":
                j += 2
            refc.append(calls[j]["counts"][0])
            confc.append(calls[j + 1]["counts"][0])
            i = j + 2
        else:
            i += 1
    return idxs, hyps, counts, refc, confc, coords


def v5_cases(RV, stub, cat_m64, cat_vertex, cat_in):
    """ransac_voting_layer_v5 as the uncertainty eval wrapper calls it
    (TRAIN:123: hn=128, inlier_thresh=0.99, max_num=100; confidence vote at
    0.999): the cat field, and a batch of two small fields (downsampled /
    fewer than min_num=5 foreground pixels)."""
    out = {}
    torch.manual_seed(31)
    stub.calls.clear()
    kp, conf = RV.ransac_voting_layer_v5(torch.from_numpy(cat_m64), torch.from_numpy(cat_vertex), 128,
                                         inlier_thresh=0.99, max_num=100)
    idxs, hyps, counts, refc, confc, coords = v5_records(stub)
    keep = np.zeros((480, 640), bool)
    keep[coords[0][:, 1].astype(int), coords[0][:, 0].astype(int)] = True
    out.update(cat_keypoints=kp.numpy(), cat_conf=conf.numpy(), cat_idxs=np.stack(idxs), cat_hyp=np.stack(hyps),
               cat_counts=np.stack(counts), cat_refine_counts=np.stack(refc), cat_conf_counts=np.stack(confc),
               cat_keep_bits=np.packbits(keep)[None], **cat_in)
    H, W = 40, 48
    fa, va = small_field(41)
    fb, vb = small_field(42, radius=1.0)                  # 5 px: min_num is 5 -> still voted? (< 5 skips)
    masks = np.stack([fa["mask"].astype(np.int64), np.zeros((H, W), np.int64)])
    masks[1, 20, 24] = 1                                  # 1 foreground pixel < min_num=5 -> zeros
    verts = np.stack([va, vb])
    torch.manual_seed(32)
    stub.calls.clear()
    kp, conf = RV.ransac_voting_layer_v5(torch.from_numpy(masks), torch.from_numpy(verts), 32,
                                         inlier_thresh=0.99, max_num=100)
    idxs, hyps, counts, refc, confc, coords = v5_records(stub)
    keep = np.zeros((2, H, W), bool)
    keep[0, coords[0][:, 1].astype(int), coords[0][:, 0].astype(int)] = True
    out.update(s_mask=masks, s_vertex=verts, s_keypoints=kp.numpy(), s_conf=conf.numpy(), s_idxs=np.stack(idxs),
               s_hyp=np.stack(hyps), s_counts=np.stack(counts), s_refine_counts=np.stack(refc),
               s_conf_counts=np.stack(confc), s_keep=keep)
    save("v5_cases", **out)


def motion_cases(RV):
    """ransac_motion_voting (RV:966-987) on offset fields: a 480x640 disk
    (29,861 px), a small field, an empty mask."""
    out = {}
    rng = np.random.default_rng(51)
    H, W, vn = 120, 160, 4
    masks = np.zeros((3, H, W), np.int64)
    yy, xx = np.mgrid[0:H, 0:W]
    masks[0] = ((xx - 80) ** 2 + (yy - 60) ** 2 <= 40 ** 2)
    masks[1] = ((xx - 30) ** 2 + (yy - 100) ** 2 <= 9 ** 2) * 2          # byte() of 2 -> foreground
    kp = rng.uniform([20, 20], [140, 100], (3, vn, 2)).astype(np.float32)
    off = kp[:, None, None] - np.stack([xx, yy], -1)[None, :, :, None].astype(np.float32)
    verts = (off + rng.normal(0, 2.0, off.shape)).astype(np.float32) * (masks != 0)[..., None, None]
    pts = RV.ransac_motion_voting(torch.from_numpy(masks), torch.from_numpy(verts)).numpy()
    out.update(mask=masks, vertex=verts, points=pts)
    save("motion_cases", **out)


def vp_kernels(stub):
    rng = np.random.default_rng(21)
    tn, vn, hn = 300, 4, 40
    direct = rng.normal(size=(tn, vn, 2)).astype(np.float32)
    coords = rng.uniform(0, 60, size=(tn, 2)).astype(np.float32).round()
    idxs = rng.integers(0, tn, size=(hn, vn, 2)).astype(np.int32)
    hyp = stub.generate_hypothesis_vanishing_point(torch.from_numpy(direct), torch.from_numpy(coords),
                                                   torch.from_numpy(idxs))
    inl = torch.zeros(hn, vn, tn, dtype=torch.uint8)
    stub.voting_for_hypothesis_vanishing_point(torch.from_numpy(direct), torch.from_numpy(coords), hyp, inl, 0.99)
    save("vp_kernels", direct=direct, coords=coords, idxs=idxs, hyp=hyp.numpy(), inliers=inl.numpy())


def main_v5():
    """Only the v5 fixtures (python tests/golden/make_golden.py v5)."""
    install_shims()
    stub = TorchKernels()
    RV = load_reference(stub)
    mask, pts3d, pose, p2d = demo_cat()
    field = synth.gt_vertex_field(mask, p2d)
    vnet = synth.to_network_layout(field)
    vertex = torch.from_numpy(vnet).permute(0, 2, 3, 1).reshape(1, 480, 640, 9, 2).numpy()
    m64 = mask.astype(np.int64)[None]
    cat_in = dict(mask_bits=np.packbits(mask.astype(bool)), points_2d=p2d, pose=pose, points_3d=pts3d,
                  field_sha=sha(field))
    v5_cases(RV, stub, m64, vertex, cat_in)


def main_motion():
    install_shims()
    RV = load_reference(TorchKernels())
    motion_cases(RV)


# YCB-Video intrinsics (lib/data_utils_xin.py:1723) and 21 keypoints per object
# (lib/datasets/YCB_dataset.py:185): BASELINE configs[4].
K_YCB = np.array([[1066.8, 0.0, 320.0], [0.0, 1066.8, 240.0], [0.0, 0.0, 1.0]])


def ycb_object():
    """21 model keypoints (a 0.12 m object) and a pose 1 m in front of the YCB
    camera; the projected keypoints fall inside the 480x640 frame."""
    rng = np.random.default_rng(2100)
    pts3d = rng.uniform(-0.06, 0.06, (21, 3))
    rv = np.array([0.4, -0.3, 0.25])
    th = np.linalg.norm(rv)
    k = rv / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    pose = np.concatenate([R, np.array([[0.01], [-0.02], [1.0]])], 1)
    return pts3d, pose, synth.project(pts3d, pose, K_YCB)


def _u16(a):
    a = np.asarray(a)
    assert a.min() >= 0 and a.max() < 65536
    return a.astype(np.uint16)


def ycb_cases(RV, stub):
    """configs[4] shapes: vn = 21 through v3 (hn 512) and EVD with mean (16 x
    256 hypotheses) on a 480x640 frame whose keypoints are the projection of
    a known pose; and the EVD branches on small frames (vn 21): a normal image,
    one with foreground < min_num (RV:343-348: zero hypotheses, ratio 1) and
    one with foreground > max_num (RV:351-355: downsampled, foreground
    re-counted), with mean and topk variants."""
    out = {}
    pts3d, pose, p2d = ycb_object()
    f = synth.synthetic_field(2101, vn=21, keypoints=p2d, center=(float(p2d[:, 0].mean()), float(p2d[:, 1].mean())))
    m = torch.argmax(torch.from_numpy(f["seg"]), 1)
    vv = torch.from_numpy(f["vertex"]).permute(0, 2, 3, 1).reshape(1, 480, 640, 21, 2)
    out.update(seed=2101, points_3d=pts3d, pose=pose, camera=K_YCB, points_2d=p2d, tn=f["tn"],
               seg_sha=sha(f["seg"]), vertex_sha=sha(f["vertex"]))
    torch.manual_seed(61)
    stub.calls.clear()
    kp = RV.ransac_voting_layer_v3(m, vv, 512, inlier_thresh=0.99).numpy()
    idxs, hyps, counts, refc, coords = per_image_records(stub)
    out.update(v3_keypoints=kp, v3_idxs=_u16(np.stack(idxs)), v3_hyp=np.stack(hyps),
               v3_counts=_u16(np.stack(counts)), v3_refine_counts=np.stack(refc),
               v3_iters=len(vote_calls(stub, "gen")))
    print("ycb v3 max err vs projection", np.abs(kp[0] - p2d).max())
    torch.manual_seed(62)
    stub.calls.clear()
    _, cov = RV.estimate_voting_distribution_with_mean(m, vv, torch.from_numpy(kp))
    gens = vote_calls(stub, "gen")
    out.update(evdm_cov=cov.numpy(), evdm_idxs=_u16(np.stack([g["idxs"] for g in gens]))[None])

    # EVD branches on 40x48 frames, vn 21
    H, W, vn = 40, 48, 21
    kin = np.random.default_rng(70).uniform([4.0, 4.0], [44.0, 36.0], (3, vn, 2))   # keypoints in the frame
    fa, va = small_field(71, vn=vn, radius=8.5, keypoints=kin[0])    # 225 px: voted as is
    fb, vb = small_field(72, vn=vn, radius=1.5, keypoints=kin[1])    # 9 px < min_num = 20 -> skipped
    fc, vc = small_field(73, vn=vn, radius=14.5, keypoints=kin[2])   # 665 px > max_num = 300 -> downsampled
    masks = np.stack([fa["mask"], fb["mask"], fc["mask"]]).astype(np.int64)
    verts = np.stack([va, vb, vc])
    means = np.stack([fa["keypoints"], fb["keypoints"], fc["keypoints"]]).astype(np.float32)
    out.update(br_mask=masks, br_vertex=verts, br_mean=means)
    for name, seed in (("mean", 63), ("topk", 64)):
        torch.manual_seed(seed)
        stub.calls.clear()
        if name == "mean":
            _, cov = RV.estimate_voting_distribution_with_mean(torch.from_numpy(masks), torch.from_numpy(verts),
                                                               torch.from_numpy(means), round_hyp_num=32,
                                                               min_hyp_num=128, max_num=300)
            out.update(br_mean_cov=cov.numpy())
        else:
            # the skipped image contributes round_hyp_num rows (RV:274), the
            # others ceil(min/round) * round_hyp_num: one round keeps the cat legal;
            # topk = all rows (ties at the k-th ratio are unspecified in torch.topk)
            mu, cov = RV.estimate_voting_distribution(torch.from_numpy(masks), torch.from_numpy(verts),
                                                      round_hyp_num=64, min_hyp_num=64, topk=64, min_num=20,
                                                      max_num=300)
            out.update(br_topk_mean=mu.numpy(), br_topk_cov=cov.numpy())
        gens = vote_calls(stub, "gen")
        per = len(gens) // 2                             # images 0 and 2 voted
        keep = np.zeros((3, H, W), bool)
        c = gens[per]["coords"]
        keep[2, c[:, 1].astype(int), c[:, 0].astype(int)] = True
        out.update({f"br_{name}_idxs": np.stack([np.stack([g["idxs"] for g in gens[:per]]),
                                                  np.stack([g["idxs"] for g in gens[per:]])]),
                    f"br_{name}_keep2": keep[2], f"br_{name}_tn": np.array([gens[0]["tn"], gens[per]["tn"]])})
    save("ycb21_cases", **out)


def main_ycb():
    install_shims()
    stub = TorchKernels()
    ycb_cases(load_reference(stub), stub)


if __name__ == "__main__":
    {"v5": main_v5, "motion": main_motion, "ycb": main_ycb}.get(sys.argv[1] if sys.argv[1:] else "", main)()
