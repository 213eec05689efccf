"""World-size-2 and -4 streams over gloo on CPU: round-robin sharding and the single
result gather of pvnet_amd.distributed, with the oracle's v3 standing in for
the device layer (the product path itself needs a GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pvnet_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _field(i):
    """Small synthetic field for image i: 48x64, 3 keypoints."""
    rng = np.random.default_rng(100 + i)
    H, W, vn = 48, 64, 3
    yy, xx = np.mgrid[0:H, 0:W]
    mask = ((xx - 32) ** 2 + (yy - 24) ** 2 < (12 + i) ** 2).astype(np.int64)
    kp = rng.uniform([20, 14], [44, 34], (vn, 2)).astype(np.float32)
    d = kp[None, None] - np.stack([xx, yy], -1)[:, :, None].astype(np.float32)
    ang = np.arctan2(d[..., 1], d[..., 0]) + rng.normal(0, 0.05, (H, W, vn))
    vertex = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32) * mask[..., None, None]
    return torch.from_numpy(mask[None]), torch.from_numpy(vertex[None])


def _oracle_vote(mask, vertex):
    from oracle import oracle as O
    kp = O.ransac_voting_layer_v3(mask.numpy(), vertex.numpy(), 32, min_num=10, seed=0)
    return torch.from_numpy(np.asarray(kp, np.float32))


def _worker(rank, world, port, n_images, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = D.run_stream(_field, _oracle_vote, n_images, rank, world, (3, 2), torch.device("cpu"))
        if rank == 0:
            np.save(out_path, res.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_round_robin():
    assert D.shard(5, 0, 2) == [0, 2, 4] and D.shard(5, 1, 2) == [1, 3]
    assert D.shard(1, 1, 2) == []
    with pytest.raises(ValueError):
        D.shard(4, 2, 2)


@pytest.mark.parametrize("world, n_images", [(2, 5), (2, 1), (4, 6), (4, 3)])
def test_stream_gloo(tmp_path, world, n_images):
    """World sizes 2 and 4 (uneven shards; a rank with no image)."""
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), n_images, out), nprocs=world, join=True)
    got = np.load(out)
    want = np.stack([_oracle_vote(*_field(i)).numpy().reshape(3, 2) for i in range(n_images)])
    np.testing.assert_array_equal(got, want)


def _multi_result(i):
    """Image i's three-part result: keypoints f32 [3, 2], covariances f32
    [3, 2, 2], pose f64 [3, 4] (values that f32 -> f64 -> f32 must keep)."""
    g = torch.Generator().manual_seed(1000 + i)
    return (torch.randn(3, 2, generator=g) * 100, torch.randn(3, 2, 2, generator=g),
            torch.randn(3, 4, generator=g, dtype=torch.float64) / 3)


def _multi_worker(rank, world, port, n_images, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = D.run_stream(lambda i: (i,), _multi_result, n_images, rank, world,
                           [(3, 2), (3, 2, 2), (3, 4)], torch.device("cpu"),
                           dtype=[torch.float32, torch.float32, torch.float64])
        if rank == 0:
            np.savez(out_path, *[r.numpy() for r in res])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world, n_images", [(2, 5), (3, 7), (2, 1)])
def test_stream_multi_result_gloo(tmp_path, world, n_images):
    """configs[4]'s stream result (keypoints, covariances, pose) gathered in
    one collective: every part comes back in stream order, dtypes and values
    unchanged."""
    out = str(tmp_path / "multi.npz")
    mp.spawn(_multi_worker, args=(world, _free_port(), n_images, out), nprocs=world, join=True)
    got = np.load(out)
    parts = [got[f"arr_{k}"] for k in range(3)]
    for i in range(n_images):
        want = _multi_result(i)
        for p, w in zip(parts, want):
            assert p.dtype == w.numpy().dtype
            np.testing.assert_array_equal(p[i], w.numpy())
