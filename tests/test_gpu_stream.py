"""configs[3] on the device: the Occlusion-LINEMOD stream (SURVEY.md 8(d)4,
BASELINE.json configs[3]) through pvnet_amd.distributed with the HIP layer.

The stream mixes full disks, occluded split disks, masks below ``min_num``
(the zeros path, RV:537-540), masks above ``max_num`` (Bernoulli
downsampling, RV:543-546; the keep-mask is drawn on the host and injected
into both sides), quadrant-occluded, empty, border-clipped and just-above-
``min_num`` masks (pvnet_amd.synth.stream_field).  Every image's hypotheses
come from injected pixel pairs, so the device counts must equal the
oracle's bit for bit and the keypoints agree to 1e-2 px.

The reference's analogue is DataParallel's scatter / gather around the
voting layer (tools/demo.py:174, tools/train_linemod.py:222-223); here one
process per rank votes its round-robin shard and one all_gather returns every
keypoint in stream order.  The two-rank test runs both ranks on cuda:0 over
gloo (RCCL refuses two ranks on one device), which covers the device-side
shard and gather code on a one-GPU box."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import oracle as O
from pvnet_amd import distributed as D
from pvnet_amd import synth

HN = 512
N_IMAGES = 16          # two cycles of the eight mask kinds
MAX_NUM, MIN_NUM = 30000, 100
KP_TOL = 1e-2


def stream_inputs(i):
    """Host inputs of stream image i: the field, its injected keep-mask and
    pixel pairs (drawn over the downsampled foreground's size)."""
    f = synth.stream_field(i)
    rng = np.random.default_rng(50_000 + i)
    keep = synth.keep_mask(f["mask"], MAX_NUM, rng)
    fg = f["mask"] & (keep != 0) if f["tn"] > MAX_NUM else f["mask"]
    tn = int(fg.sum())
    idxs = rng.integers(0, max(tn, 1), (1, HN, 9, 2)).astype(np.int32)
    return f, keep[None], idxs


def oracle_image(f, keep, idxs):
    vv = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
    dg = []
    kp = O.ransac_voting_layer_v3(np.argmax(f["seg"], 1), vv, HN, min_num=MIN_NUM, max_num=MAX_NUM,
                                  idxs=[idxs[0]], keep=keep, diag=dg)
    return kp[0], dg[0]


def make_vote(ws, diags):
    from pvnet_amd import ransac_voting_gpu as rvg

    def vote(seg, ver, idxs, keep, i):
        d = {}
        kp = rvg.ransac_voting_layer_v3_from_network(seg, ver, HN, min_num=MIN_NUM, max_num=MAX_NUM, _idxs=idxs,
                                                     _keep=keep, _diag=d, _workspace=ws)
        diags[i] = d
        return kp
    return vote


def make_load(dev):
    def load(i):
        f, keep, idxs = stream_inputs(i)
        return (torch.from_numpy(f["seg"]).to(dev), torch.from_numpy(f["vertex"]).to(dev),
                torch.from_numpy(idxs).to(dev), torch.from_numpy(keep).to(dev), i)
    return load


def check_against_oracle(kps, diags):
    kinds = set()
    for i in range(N_IMAGES):
        f, keep, idxs = stream_inputs(i)
        ko, dg = oracle_image(f, keep, idxs)
        kinds.add(f["kind"])
        if dg.get("skipped"):
            assert f["tn"] < MIN_NUM, (i, f["kind"])
            if diags is not None:
                assert int(diags[i]["tn"].cpu()[0]) == 0, (i, f["kind"])
            assert np.all(kps[i] == 0), (i, f["kind"])
            continue
        if diags is not None:
            d = {k: v.cpu().numpy() for k, v in diags[i].items()}
            assert int(d["tn"][0]) == dg["tn"], (i, f["kind"])
            np.testing.assert_array_equal(d["counts"][0].T, dg["counts"], err_msg=f"image {i} ({f['kind']})")
            np.testing.assert_array_equal(d["win_idx"][0], dg["win_idx"], err_msg=f"image {i} ({f['kind']})")
        np.testing.assert_allclose(kps[i], ko, atol=KP_TOL, rtol=0, err_msg=f"image {i} ({f['kind']})")
    assert kinds == set(synth.STREAM_KINDS)


def test_stream_kinds_cover_config3_cases():
    """The stream holds each case SURVEY 8(d)4 names (a cheap host check)."""
    tns = {}
    for i in range(8):
        f = synth.stream_field(i)
        tns[f["kind"]] = f["tn"]
    assert tns["full"] == 29861
    assert 0 < tns["tiny"] < MIN_NUM and tns["empty"] == 0
    assert tns["large"] > MAX_NUM
    assert MIN_NUM <= tns["small"] < 400
    split = synth.stream_field(1)["mask"]
    cols = np.nonzero(split.any(0))[0]
    assert np.any(np.diff(cols) > 1), "the occluder splits the disk in two"


@pytest.mark.gpu
def test_config3_stream_one_rank(device):
    """One rank: D.run_stream over the HIP layer, every image against the oracle."""
    from pvnet_amd import ransac_voting_gpu as rvg
    diags = {}
    res = D.run_stream(make_load(device), make_vote(rvg.VotingWorkspace(), diags), N_IMAGES, 0, 1, (9, 2), device)
    check_against_oracle(res.cpu().numpy(), diags)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, out_path):
    import torch.distributed as dist
    from pvnet_amd import ransac_voting_gpu as rvg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        diags = {}
        res = D.run_stream(make_load(dev), make_vote(rvg.VotingWorkspace(), diags), N_IMAGES, rank, world, (9, 2),
                           dev)
        assert res.device == dev and res.shape == (N_IMAGES, 9, 2)
        # this rank's own images came back to their stream slots unchanged
        mine = D.shard(N_IMAGES, rank, world)
        for i in mine:
            d = diags[i]
            if int(d["tn"].cpu()[0]) == 0:
                assert torch.all(res[i] == 0)
        np.save(out_path + f".{rank}.npy", res.cpu().numpy())
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config3_stream_two_ranks_gloo(device, tmp_path):
    """World size 2, both ranks on cuda:0 running the HIP layer on their
    round-robin shards, one gather: every rank holds the whole stream in
    order, equal to the oracle's keypoints."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "res")
    mp.spawn(_rank_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(r0, r1)
    check_against_oracle(r0, None)


# ---------------------------------------------------------------- configs[4]: keypoints + covariances + poses
# The YCB-Video stream (BASELINE.json configs[4]): per image ransac_voting_layer_v3
# (hn 512) from the network layout, estimate_voting_distribution_with_mean
# (16 x 256 hypotheses, RV:333-406) on argmax(seg) and the strided vertex view,
# and the uncertainty PnP of the 21 keypoints (evaluation_utils.py:161-190);
# the stream is sharded round-robin and (keypoints [21, 2], covariances
# [21, 2, 2], pose [3, 4]) come back in one gather (the [vn, 2, 2] payload of
# SURVEY 8(e)).  Even images are the golden ycb21 frame (the reference's own
# keypoints and covariances, its idxs injected); odd ones are 21-keypoint
# fields projected from random poses through the YCB camera (checked against
# the oracle's v3 -> EVD -> PnP with the same injected idxs).
N4 = 4
COV4_RTOL = 1e-4


def ycb_stream_inputs(i):
    from tests import golden_io as G
    g = G.load("ycb21_cases")
    K, p3 = g["camera"], g["points_3d"]
    if i % 2 == 0:
        _, _, f = G.ycb_inputs(g)
        i3 = g["v3_idxs"].astype(np.int32)
        i4 = g["evdm_idxs"].astype(np.int32).reshape(1, -1, 21, 2)
        return f, i3, i4, g
    rng = np.random.default_rng(70_000 + i)
    a = rng.normal(size=3) * 0.5
    th = np.linalg.norm(a)
    kx = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]) / th
    R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
    X = p3 @ R.T + np.array([rng.uniform(-0.05, 0.05), rng.uniform(-0.05, 0.05), rng.uniform(0.9, 1.1)])
    kp = np.stack([K[0, 0] * X[:, 0] / X[:, 2] + K[0, 2], K[1, 1] * X[:, 1] / X[:, 2] + K[1, 2]], 1)
    f = synth.synthetic_field(7000 + i, vn=21, keypoints=kp, radius=40.0,
                              center=(float(kp[:, 0].mean()), float(kp[:, 1].mean())))
    tn = int(f["tn"])
    i3 = rng.integers(0, tn, (1, HN, 21, 2)).astype(np.int32)
    i4 = rng.integers(0, tn, (1, 16 * 256, 21, 2)).astype(np.int32)
    return f, i3, i4, None


def ycb_expected(i):
    """(keypoints, covariances, pose) the stream must return for image i."""
    from oracle import pnp as P
    f, i3, i4, g = ycb_stream_inputs(i)
    from tests import golden_io as G
    gg = G.load("ycb21_cases")
    K, p3 = gg["camera"], gg["points_3d"]
    if g is not None:
        kp, cov = g["v3_keypoints"][0], g["evdm_cov"][0]
    else:
        mask = np.argmax(f["seg"], 1)
        vv = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, 480, 640, 21, 2))
        kp = O.ransac_voting_layer_v3(mask, vv, HN, idxs=[i3[0]])
        _, cov = O.estimate_voting_distribution_with_mean(mask, vv, kp, idxs=[list(i4[0].reshape(16, 256, 21, 2))])
        kp, cov = kp[0], cov[0]
    return kp, cov, P.uncertainty_pnp(kp, P.weights_from_cov(cov), p3, K)


def make_vote4(dev):
    from pvnet_amd import extend_utils as eu
    from pvnet_amd import ransac_voting_gpu as rvg
    from tests import golden_io as G
    gg = G.load("ycb21_cases")
    K, p3 = gg["camera"], gg["points_3d"]
    w1, w2 = rvg.VotingWorkspace(), rvg.VotingWorkspace()

    def load(i):
        f, i3, i4, _ = ycb_stream_inputs(i)
        return (torch.from_numpy(f["seg"]).to(dev), torch.from_numpy(f["vertex"]).to(dev),
                torch.from_numpy(i3).to(dev), torch.from_numpy(i4).to(dev))

    def vote(seg, ver, i3, i4):
        b, c, h, w = ver.shape
        kp = rvg.ransac_voting_layer_v3_from_network(seg, ver, HN, _idxs=i3, _workspace=w1)
        mask = seg.argmax(1)
        vertex = ver.permute(0, 2, 3, 1).view(b, h, w, c // 2, 2)
        mean, cov = rvg.estimate_voting_distribution_with_mean(mask, vertex, kp, _idxs=i4, _workspace=w2)
        Rt = eu.pose_from_voting(mean, cov, p3, K)
        return kp[0], cov[0], Rt[0]
    return load, vote


def check_ycb_stream(res):
    kps, covs, poses = (r.cpu().numpy() for r in res)
    assert kps.shape == (N4, 21, 2) and covs.shape == (N4, 21, 2, 2) and poses.shape == (N4, 3, 4)
    assert poses.dtype == np.float64
    for i in range(N4):
        kp, cov, pose = ycb_expected(i)
        np.testing.assert_allclose(kps[i], kp, atol=KP_TOL, rtol=0, err_msg=f"image {i}")
        np.testing.assert_allclose(covs[i], cov, rtol=COV4_RTOL, atol=1e-4 * np.abs(cov).max(), err_msg=f"image {i}")
        np.testing.assert_allclose(poses[i], pose, atol=1e-4, err_msg=f"image {i}")


@pytest.mark.gpu
def test_config4_stream_one_rank(device):
    """configs[4] on one rank: keypoints, covariances and poses of every image."""
    load, vote = make_vote4(device)
    res = D.run_stream(load, vote, N4, 0, 1, [(21, 2), (21, 2, 2), (3, 4)], device,
                       dtype=[torch.float32, torch.float32, torch.float64])
    check_ycb_stream(res)


def _rank_worker4(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        load, vote = make_vote4(dev)
        res = D.run_stream(load, vote, N4, rank, world, [(21, 2), (21, 2, 2), (3, 4)], dev,
                           dtype=[torch.float32, torch.float32, torch.float64])
        assert all(r.device == dev for r in res)
        np.savez(out_path + f".{rank}.npz", *[r.cpu().numpy() for r in res])
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config4_stream_two_ranks_gloo(device, tmp_path):
    """configs[4] sharded over two ranks (both on cuda:0, gloo): each rank
    votes, estimates the covariances and solves the poses of its round-robin
    shard; one gather gives every rank the whole stream's keypoints,
    covariances and poses in order, equal to the reference's / the oracle's."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "res4")
    mp.spawn(_rank_worker4, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = np.load(out + ".0.npz"), np.load(out + ".1.npz")
    for k in r0.files:
        np.testing.assert_array_equal(r0[k], r1[k])
    check_ycb_stream([torch.from_numpy(r0[f"arr_{k}"]) for k in range(3)])


def _rccl_worker(rank, port, out_path):
    """One rank over the nccl backend (RCCL on ROCm) with the device given at
    init, as bench.py's multi-GPU ranks start: the stream's gather then runs
    RCCL's all_gather_into_tensor on device tensors (a one-rank copy, but the
    same backend, communicator setup and device-tensor path an 8-GPU run
    takes; RCCL refuses two ranks on one device)."""
    import torch.distributed as dist
    from pvnet_amd import ransac_voting_gpu as rvg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        diags = {}
        res = D.run_stream(make_load(dev), make_vote(rvg.VotingWorkspace(), diags), N_IMAGES, 0, 1, (9, 2), dev)
        assert res.device == dev and res.shape == (N_IMAGES, 9, 2)
        kp, cov = torch.randn(5, 9, 2, device=dev), torch.randn(5, 9, 2, 2, device=dev)
        pose = torch.randn(5, 3, 4, device=dev, dtype=torch.float64)
        g = D.gather_results_multi([kp, cov, pose], 5, 0, 1)
        assert all(x.device == dev for x in g)
        assert torch.equal(g[0], kp) and torch.equal(g[1], cov) and torch.equal(g[2], pose)
        np.save(out_path + ".npy", res.cpu().numpy())
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config3_stream_rccl_one_rank(device, tmp_path):
    """The nccl (RCCL) backend's gather path on the device: every keypoint in
    stream order, equal to the oracle's."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "rccl")
    mp.spawn(_rccl_worker, args=(_free_port(), out), nprocs=1, join=True)
    check_against_oracle(np.load(out + ".npy"), None)
