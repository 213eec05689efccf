"""Multi-GPU stream of images through the voting path.

Images are independent (the reference's per-image loops RV:531, RV:337), so
the stream shards with no data-path collective: image i goes to rank
``i % world`` (round-robin), every rank runs the whole vote -> keypoint path
on its own images with device-resident inputs, and the only exchange is one
gather of the results to rank 0 at the end of a stream chunk -- 72 B of
keypoints per image (plus 64 B of covariance when EVD runs), so it is
latency-bound and happens once per chunk.  On ROCm the ``nccl`` backend is
RCCL over xGMI; the CPU tests run the same code over ``gloo``.

This replaces the reference's ``DataParallel`` scatter / gather around the
voting layer (DEMO:174, tools/parallel.py:183-200): one process per GPU, no
threads, no GIL contention.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

__all__ = ["shard", "gather_results", "gather_results_multi", "run_stream"]


def shard(n_images: int, rank: int, world: int) -> list[int]:
    """Round-robin image indices of ``rank`` (image i -> rank i % world)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return list(range(rank, n_images, world))


def gather_results(local: torch.Tensor, n_images: int, rank: int, world: int,
                   group: Optional[dist.ProcessGroup] = None) -> Optional[torch.Tensor]:
    """Reassemble per-rank results in stream order on every rank.

    ``local`` is ``[len(shard(n_images, rank, world)), ...]`` in shard order.
    Ranks hold ``ceil`` or ``floor`` of n_images / world rows; the tensors are
    padded to the ceiling so one ``all_gather_into_tensor`` moves them all.
    Returns ``[n_images, ...]`` (row i = image i).
    """
    per = (n_images + world - 1) // world
    feat = tuple(local.shape[1:])
    grouped = dist.is_available() and dist.is_initialized()
    if grouped and dist.get_world_size(group) != world:
        if world != 1:
            raise ValueError(f"world {world} differs from the process group's size {dist.get_world_size(group)}")
        grouped = False     # a local-only gather inside a multi-rank job
    if world == 1 and not grouped:
        return local        # nothing to exchange (in a one-rank group the collective runs: a copy)
    if local.shape[0] != len(range(rank, n_images, world)):
        raise ValueError(f"rank {rank} holds {local.shape[0]} results, its shard has {len(range(rank, n_images, world))}")
    # RCCL moves device tensors over xGMI; gloo (the CPU tests, or ranks that
    # share one device) exchanges host copies -- the collective only, the
    # results stay where the caller's device put them
    stage = local.device.type == "cuda" and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if stage else local.device
    pad = torch.zeros((per,) + feat, dtype=local.dtype, device=dev)
    pad[:local.shape[0]] = local
    allv = torch.empty((world * per,) + feat, dtype=local.dtype, device=dev)
    dist.all_gather_into_tensor(allv, pad, group=group)
    allv = allv.view((world, per) + feat)
    # image i = rank i % world, slot i // world
    idx = torch.arange(n_images, device=dev)
    out = allv[idx % world, idx // world]
    return out.to(local.device) if stage else out


def gather_results_multi(parts: Sequence[torch.Tensor], n_images: int, rank: int, world: int,
                         group: Optional[dist.ProcessGroup] = None) -> tuple:
    """:func:`gather_results` for a result of several tensors per image (the
    configs[4] stream: keypoints [vn, 2] f32, covariances [vn, 2, 2] f32,
    pose [3, 4] f64).  Each part is ``[len(shard), *shape_k]``; they travel
    as one f64 row per image (every f32 is exact in f64), so one collective
    moves them all.  Returns a tuple of ``[n_images, *shape_k]`` in stream
    order, each in its part's dtype."""
    n = int(parts[0].shape[0])
    if any(int(p.shape[0]) != n for p in parts):
        raise ValueError("every part needs one row per image of the shard")
    sizes = [int(torch.Size(p.shape[1:]).numel()) for p in parts]
    flat = torch.cat([p.reshape(n, k).to(torch.float64) for p, k in zip(parts, sizes)], 1)
    allf = gather_results(flat, n_images, rank, world, group)
    out, o = [], 0
    for p, k in zip(parts, sizes):
        out.append(allf[:, o:o + k].reshape((n_images,) + tuple(p.shape[1:])).to(p.dtype))
        o += k
    return tuple(out)


def run_stream(load: Callable[[int], Sequence[torch.Tensor]], vote: Callable[..., torch.Tensor], n_images: int,
               rank: int, world: int, result_shape, device: torch.device,
               dtype=torch.float32, group: Optional[dist.ProcessGroup] = None):
    """Vote every image of this rank's shard, then gather all results.

    ``load(i)`` returns the arguments of ``vote`` for image i (already on
    this rank's device); ``vote(*args)`` returns that image's result of
    ``result_shape`` (e.g. ``ransac_voting_layer_v3_from_network`` ->
    ``[1, vn, 2]`` with result_shape ``(vn, 2)``).  Returns
    ``[n_images, *result_shape]`` in stream order on every rank.

    A result of several tensors (e.g. keypoints, covariances and the pose of
    configs[4]): ``vote`` returns a tuple, ``result_shape`` is a list of
    shapes and ``dtype`` a list of dtypes; the return value is then a tuple
    (:func:`gather_results_multi`).
    """
    mine = shard(n_images, rank, world)
    multi = len(result_shape) > 0 and isinstance(result_shape[0], (tuple, list, torch.Size))
    if not multi:
        local = torch.empty((len(mine),) + tuple(result_shape), dtype=dtype, device=device)
        for k, i in enumerate(mine):
            local[k] = vote(*load(i)).reshape(tuple(result_shape))
        return gather_results(local, n_images, rank, world, group)
    dtypes = list(dtype) if isinstance(dtype, (tuple, list)) else [dtype] * len(result_shape)
    locals_ = [torch.empty((len(mine),) + tuple(sh), dtype=dt, device=device)
               for sh, dt in zip(result_shape, dtypes)]
    for k, i in enumerate(mine):
        res = vote(*load(i))
        if len(res) != len(locals_):
            raise ValueError(f"vote returned {len(res)} tensors, result_shape names {len(locals_)}")
        for loc, r, sh in zip(locals_, res, result_shape):
            loc[k] = r.reshape(tuple(sh))
    return gather_results_multi(locals_, n_images, rank, world, group)
