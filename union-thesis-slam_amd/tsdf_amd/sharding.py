"""Multi-GPU partitioning of the fusion path, one process per GPU.

Dense grid: rank r of N owns the x-slab [x0, x1) of the volume (x is the slowest axis of the
reference's C-order (X,Y,Z) layout, grid_fusion.py:52-55, so a slab is contiguous there).  Every
rank integrates every frame into its slab; world coordinates come from the GLOBAL voxel index,
so the slabs are bit-identical to the same voxels of one unsharded volume and no data moves
between GPUs while integrating.  Only get_volume gathers the slabs.

Voxel hash: rank r owns the 8^3 blocks whose home slot (the reference's hash_function of the block
coordinates, hash_fusion.py:182-190) falls in [r*n/N, (r+1)*n/N) of the n-slot table (SURVEY.md
§8(e)).  Again every rank sees every frame and the block sets are disjoint; the dense export
merges them.

Collectives (torch.distributed: RCCL "nccl" on the GPU box, "gloo" in the CPU tests) appear only
outside the integrate loop: gathering the slabs / merging the hash exports and summing counters.
"""
from __future__ import annotations

import numpy as np

BRICK = 8
P1, P2, P3 = 73856093, 19349669, 83492791


def slab(rank: int, world: int, nx: int, align: int = BRICK):
    """[x0, x1) of `rank`: near-equal shares of nx voxels, cut on brick boundaries when the
    volume is large enough so that no brick straddles two ranks."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    if nx >= align * world:
        nb = -(-nx // align)
        b0, b1 = rank * nb // world, (rank + 1) * nb // world
        return min(nx, b0 * align), min(nx, b1 * align)
    return rank * nx // world, (rank + 1) * nx // world


def columns(rank: int, world: int, nx: int):
    """Global x indices owned by `rank` under cyclic brick-column sharding (the layout
    tsdf_dense_create_shard builds): the 8-voxel x-columns c with c % world == rank, in order.
    Every rank then sees a similar share of each frame's frustum, unlike contiguous slabs."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    x = np.arange(nx, dtype=np.int64)
    own = x[(x // BRICK) % world == rank]
    if own.size == 0:
        raise ValueError(f"rank {rank} of {world} owns no 8-voxel column of {nx}")
    return own


def ref_hash(x, y, z, n: int, int_bits: int = 64):
    """hash_function (hash_fusion.py:182-190) on integer arrays: int64 or wrapping-int32 mode."""
    x, y, z = (np.asarray(a, dtype=np.int64) for a in (x, y, z))
    with np.errstate(over="ignore"):
        if int_bits == 32:
            h = (x * P1).astype(np.int32) ^ (y * P2).astype(np.int32) ^ (z * P3).astype(np.int32)
            h = h.astype(np.int64)
        else:
            h = (x * P1) ^ (y * P2) ^ (z * P3)
    return np.remainder(h, n)


def hash_owner(bx, by, bz, capacity: int, n_shards: int, int_bits: int = 64):
    """Shard owning block (bx,by,bz): the bucket range its home slot falls in (the same
    arithmetic as k_cull<true>).  `capacity` is the table's capacity at create: ownership is
    fixed then (Table::shard_cap) and does not follow later resizes, so no block ever moves
    between shards."""
    home = ref_hash(bx, by, bz, capacity, int_bits)
    return (home * n_shards) // capacity


def gather_slabs(local: np.ndarray, x_range, nx: int, group=None, dst: int = 0):
    """Assemble x-slabs of an (x, Y, Z) array on rank `dst` (None elsewhere)."""
    return gather_rows(local, np.arange(x_range[0], x_range[1], dtype=np.int64), nx, group, dst)


def gather_rows(local: np.ndarray, x_index, nx: int, group=None, dst: int = 0):
    """Assemble the x rows of an (x, Y, Z) array, local row i being global row x_index[i]
    (slabs or cyclic columns), on rank `dst` (None elsewhere)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    x_index = np.asarray(x_index, dtype=np.int64)
    if len(x_index) != local.shape[0]:
        raise ValueError("x_index length differs from the local x extent")
    t = torch.from_numpy(np.ascontiguousarray(local)).reshape(-1)
    rows = torch.full((nx,), -1, dtype=torch.int64)
    rows[: len(x_index)] = torch.from_numpy(x_index)
    n_rows = [torch.zeros(nx, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(n_rows, rows, group=group)
    row = int(np.prod(local.shape[1:], dtype=np.int64))
    n_max = max(int((r >= 0).sum()) for r in n_rows) * row
    buf = torch.zeros(n_max, dtype=t.dtype)
    buf[: t.numel()] = t
    parts = [torch.zeros(n_max, dtype=t.dtype) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    if rank != dst:
        return None
    out = np.empty((nx,) + local.shape[1:], dtype=local.dtype)
    seen = np.zeros(nx, dtype=np.int64)
    for r_idx, p in zip(n_rows, parts):
        xi = r_idx.numpy()
        xi = xi[xi >= 0]
        out[xi] = p[: len(xi) * row].numpy().reshape((len(xi),) + local.shape[1:])
        seen[xi] += 1
    if not (seen == 1).all():
        raise RuntimeError("x rows missing or owned twice across ranks")
    return out


def merge_hash_exports(tsdf, weight, color, group=None):
    """Merge per-shard dense exports (disjoint voxel sets: a voxel is owned where its weight
    is > 0) into the full volume on every rank."""
    import torch
    import torch.distributed as dist

    w = torch.from_numpy(np.ascontiguousarray(weight))
    own = (w > 0)
    t = torch.where(own, torch.from_numpy(np.ascontiguousarray(tsdf)), torch.zeros_like(w))
    c = torch.where(own, torch.from_numpy(np.ascontiguousarray(color)), torch.zeros_like(w))
    cnt = own.to(torch.int32)
    for x in (w, t, c, cnt):
        dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    if int(cnt.max()) > 1:
        raise RuntimeError("hash shards overlap: a voxel is owned by more than one rank")
    t = torch.where(cnt > 0, t, torch.ones_like(t))
    return t.numpy(), w.numpy(), c.numpy()


def sum_counters(d: dict, group=None) -> dict:
    """All-reduce (sum) a dict of integer counters."""
    import torch
    import torch.distributed as dist

    keys = sorted(k for k, v in d.items() if isinstance(v, (int, np.integer)))
    t = torch.tensor([int(d[k]) for k in keys], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}
