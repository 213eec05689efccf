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
