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

Collectives (torch.distributed: RCCL "nccl" on the GPU box with device tensors, "gloo" on host
tensors in the CPU tests) appear only outside the integrate loop: the device-side gather of the
rows for get_volume, the point-to-point exchange of border rows for sharded marching cubes (the
"border-slab" step of BASELINE config[3]: halo copies are identical on both sides, so the
"reduce" is a select), the sparse block merge of hash shards, and counter sums.
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
    tsdf_dense_create_shard builds): in every period of 2*world 8-voxel x-columns, columns rank
    and 2*world-1-rank (mirrored pairs), in order.  Every rank then sees a similar share of each
    frame's frustum, unlike contiguous slabs, and a work density drifting along x evens out."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    x = np.arange(nx, dtype=np.int64)
    ph = (x // BRICK) % (2 * world)
    own = x[(ph == rank) | (ph == 2 * world - 1 - rank)]
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
    arithmetic as k_cull<true>).  `capacity` is the table size at create (map_size); the device
    table has S = the power of two >= it slots and the home slot is the hash floor-mod S.
    Ownership is fixed at create (Table::shard_cap) and does not follow later resizes, so no
    block ever moves between shards."""
    slots = 1 << (int(capacity) - 1).bit_length()
    home = ref_hash(bx, by, bz, slots, int_bits)
    return (home * n_shards) // slots


_BUFFER_DEVICE = None


def set_buffer_device(device):
    """Override where collective buffers live (None: by backend, _device).  The GPU tests' 2-rank
    job runs gloo with device buffers ("cuda"), so the branches the RCCL run takes -- rows read
    into device tensors, halos and blocks handed to the library as device pointers -- execute on
    the one-GPU box too; gloo moves device tensors itself for broadcast, all_reduce and
    all_gather, and through host copies for gather and point-to-point (_gloo_staged)."""
    global _BUFFER_DEVICE
    _BUFFER_DEVICE = device


def _device(group=None):
    """Where collective buffers live: the rank's GPU under RCCL ("nccl"), host memory under gloo
    (the CPU tests), or the set_buffer_device override."""
    import torch
    import torch.distributed as dist
    if _BUFFER_DEVICE is not None:
        d = torch.device(_BUFFER_DEVICE)
        return torch.device("cuda", torch.cuda.current_device()) if d.type == "cuda" and d.index is None else d
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _gloo_staged(group=None):
    """Device buffers on gloo: gather and point-to-point go through host copies (gloo has no
    device-tensor path for them); RCCL takes the device tensors directly."""
    import torch.distributed as dist
    return _device(group).type == "cuda" and dist.get_backend(group) == "gloo"


def _all_x_index(x_index, group=None):
    """Every rank's global x rows (list indexed by rank)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, [int(v) for v in x_index], group=group)
    return [np.asarray(o, dtype=np.int64) for o in out]


def gather_slabs(local: np.ndarray, x_range, nx: int, group=None, dst: int = 0):
    """Assemble x-slabs of an (x, Y, Z) array on rank `dst` (None elsewhere)."""
    return gather_rows(local, np.arange(x_range[0], x_range[1], dtype=np.int64), nx, group, dst)


def gather_rows(local, x_index, nx: int, group=None, dst: int = 0):
    """Assemble the x rows of an (x, Y, Z) array, local row i being global row x_index[i]
    (slabs or cyclic columns), on rank `dst` (None elsewhere).  `local` is a numpy array or a
    tensor; the rows travel in the backend's memory (device tensors under RCCL)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _device(group)
    x_index = np.asarray(x_index, dtype=np.int64)
    t = local if isinstance(local, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(local))
    t = t.to(dev)
    if len(x_index) != t.shape[0]:
        raise ValueError("x_index length differs from the local x extent")
    rows_all = _all_x_index(x_index, group)
    row = int(np.prod(t.shape[1:], dtype=np.int64))
    n_max = max(len(r) for r in rows_all) * row
    buf = torch.zeros(n_max, dtype=t.dtype, device=dev)
    buf[: t.numel()] = t.reshape(-1)
    parts = [torch.empty(n_max, dtype=t.dtype, device=dev) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    if rank != dst:
        return None
    seen = np.zeros(nx, dtype=np.int64)
    out = torch.empty((nx,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    for xi, p in zip(rows_all, parts):
        out[torch.from_numpy(xi).to(dev)] = p[: len(xi) * row].reshape((len(xi),) + tuple(t.shape[1:]))
        seen[xi] += 1
    if not (seen == 1).all():
        raise RuntimeError("x rows missing or owned twice across ranks")
    return out.cpu().numpy()


def gather_volume(vol, group=None, dst: int = 0, weight: bool = True):
    """get_volume of a sharded TSDFVolume (grid_fusion.py:316-320): every rank reads its rows
    straight from its brick layout into device buffers (tsdf_dense_get_rows), RCCL all-gathers
    them, rank `dst` scatters them into the (X, Y, Z) volume on its GPU and copies it to the host
    once.  Returns (tsdf, weight, colour) numpy arrays on `dst`, None elsewhere."""
    import torch
    dev = _device(group)
    n = len(vol.x_index)
    shape = (n, int(vol._local_dim[1]), int(vol._local_dim[2]))
    if dev.type == "cuda":
        torch.cuda.synchronize()
        bufs = [torch.empty(shape, dtype=torch.float32, device=dev) if (k != 1 or weight) else None for k in range(3)]
        vol.get_rows(np.arange(n), out=bufs)
    else:
        t, w, c = vol.get_rows(np.arange(n), weight=weight)
        bufs = [torch.from_numpy(t), None if w is None else torch.from_numpy(w), torch.from_numpy(c)]
    X = int(vol._vol_dim[0])
    out = [None if b is None else gather_rows(b, vol.x_index, X, group, dst) for b in bufs]
    return tuple(out) if out[0] is not None else None


def exchange_halo(vol, group=None):
    """The border rows each shard's marching cubes needs from its neighbours
    (tsdf_dense_mesh_halo_rows), exchanged point to point: every rank reads the rows the others
    need from its brick layout into one buffer (tsdf_dense_get_rows) and the pairs trade them
    with batched isend / irecv (device tensors over xGMI under RCCL).  Returns (global x (n,),
    tsdf (n,Y,Z), colour (n,Y,Z)) in this rank's memory for TSDFVolume.extract_mesh(halo=...)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _device(group)
    staged = _gloo_staged(group)
    X = int(vol._vol_dim[0])
    Y, Z = int(vol._local_dim[1]), int(vol._local_dim[2])
    need = vol.mesh_halo_rows(X)
    owners = _all_x_index(vol.x_index, group)
    owner_of = np.full(X, -1, np.int64)
    for r, xi in enumerate(owners):
        owner_of[xi] = r
    needs = [None] * world
    dist.all_gather_object(needs, [int(v) for v in need], group=group)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    local_row = {int(g): i for i, g in enumerate(vol.x_index)}
    ops, recv = [], {}
    for p in range(world):
        if p == rank:
            continue
        give = [g for g in needs[p] if owner_of[g] == rank]  # rows p needs from me
        take = [g for g in need if owner_of[g] == p]          # rows I need from p
        if give:
            lr = np.array([local_row[g] for g in give], np.int64)
            if dev.type == "cuda":
                sb = torch.empty((2, len(lr), Y, Z), dtype=torch.float32, device=dev)
                vol.get_rows(lr, out=[sb[0], None, sb[1]])
                torch.cuda.synchronize()
                if staged:
                    sb = sb.cpu()
            else:
                t, _, c = vol.get_rows(lr, weight=False)
                sb = torch.from_numpy(np.stack([t, c]))
            ops.append(dist.P2POp(dist.isend, sb, p, group=group))
        if take:
            rb = torch.empty((2, len(take), Y, Z), dtype=torch.float32, device="cpu" if staged else dev)
            recv[p] = (take, rb)
            ops.append(dist.P2POp(dist.irecv, rb, p, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if staged:
        recv = {p: (tk, rb.to(dev)) for p, (tk, rb) in recv.items()}
    if dev.type == "cuda":
        torch.cuda.synchronize()
    missing = [g for g in need if owner_of[g] < 0]
    if missing:
        raise RuntimeError(f"halo rows {missing[:4]} are owned by no rank")
    gx = np.concatenate([np.asarray(recv[p][0], np.int64) for p in sorted(recv)]) if recv else np.zeros(0, np.int64)
    if not recv:
        return gx, None, None
    order = np.argsort(gx, kind="stable")  # rows in increasing x
    gx = gx[order]
    sel = torch.from_numpy(order).to(dev)
    ht = torch.cat([recv[p][1][0] for p in sorted(recv)])[sel]
    hc = torch.cat([recv[p][1][1] for p in sorted(recv)])[sel]
    if dev.type == "cpu":
        ht, hc = ht.numpy(), hc.numpy()
    else:
        ht, hc = ht.contiguous(), hc.contiguous()
    return gx, ht, hc


def mesh_shard(vol, group=None):
    """Marching cubes of one shard with its halo (exchange_halo): the cells anchored at the
    shard's own rows, vertices carrying their global keys.  Returns (verts, faces, normals,
    colors, keys) numpy arrays; merge_meshes unites the shards' meshes."""
    gx, ht, hc = exchange_halo(vol, group)
    v, n, c, f, k = vol.extract_mesh(halo=(gx, ht, hc) if ht is not None else None,
                                     global_x=int(vol._vol_dim[0]), keys=True)
    return v, f, n, c, k


def merge_meshes(parts):
    """Union of shard meshes (verts, faces, normals, colors, keys): vertices merged by global key
    (the copies of a border vertex are bit-identical), ordered by key like the unsharded mesh's
    (voxel, axis) C-order; faces re-indexed.  Returns (verts, faces, normals, colors)."""
    keys = np.concatenate([p[4] for p in parts])
    uk, first = np.unique(keys, return_index=True)
    verts = np.concatenate([p[0] for p in parts])[first]
    norms = np.concatenate([p[2] for p in parts])[first]
    cols = np.concatenate([p[3] for p in parts])[first]
    faces = [np.searchsorted(uk, p[4][p[1]]).astype(np.int32) for p in parts if len(p[1])]
    faces = np.concatenate(faces) if faces else np.zeros((0, 3), np.int32)
    return verts, faces, norms, cols


def gather_meshes(part, group=None, dst: int = 0):
    """All shards' meshes on rank `dst`, merged (merge_meshes); None elsewhere."""
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group) if dist.get_rank(group) == dst else None
    dist.gather_object(part, parts, dst=dst, group=group)
    return merge_meshes(parts) if parts is not None else None


def merge_hash_shards(ht, make_table, group=None, dst: int = 0):
    """Merge bucket-range hash shards (disjoint block sets) into one table on rank `dst`: each rank
    exports only its live blocks (tsdf_hash_export_blocks, device buffers under RCCL), the blocks
    are gathered to `dst` and imported into `make_table()` (an unsharded HashTable).  Ownership is
    carried by the blocks themselves, so entries with weight 0 survive.  Returns the merged table
    on `dst`, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _device(group)
    if dev.type == "cuda":
        torch.cuda.synchronize()
        blocks = ht.export_blocks(device=dev)
    else:
        blocks = [torch.from_numpy(b.view(np.int64) if b.dtype == np.uint64 else b) for b in ht.export_blocks()]
    cnt = torch.tensor([blocks[0].shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    n_max = max(counts)
    merged = make_table() if rank == dst else None
    fields = []
    staged = _gloo_staged(group)
    for b in blocks:  # one field at a time keeps the padded buffers small
        pad = torch.zeros((n_max,) + tuple(b.shape[1:]), dtype=b.dtype, device=dev)
        pad[: b.shape[0]] = b
        if staged:
            pad = pad.cpu()
        got = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, got, dst=dst, group=group)
        if rank == dst:
            fields.append(torch.cat([g[:c] for g, c in zip(got, counts)]).to(dev))
    if rank != dst:
        return None
    if dev.type == "cuda":
        torch.cuda.synchronize()
        merged.import_blocks(fields[0], fields[1], fields[2], fields[3], fields[4])
    else:
        arr = [f.numpy() for f in fields]
        merged.import_blocks(arr[0], arr[1], arr[2], arr[3], arr[4].view(np.uint64))
    return merged


def merge_hash_exports(tsdf, weight, color, group=None):
    """Merge per-shard dense exports (disjoint voxel sets: a voxel is owned where its weight
    is > 0) into the full volume on every rank.  Dense and host-side: kept for small volumes;
    merge_hash_shards moves only live blocks."""
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
    """All-reduce (sum) a dict of integer counters (in the backend's memory)."""
    import torch
    import torch.distributed as dist

    keys = sorted(k for k, v in d.items() if isinstance(v, (int, np.integer)))
    t = torch.tensor([int(d[k]) for k in keys], dtype=torch.int64, device=_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def broadcast_frames(depth, rgb, Tinv, group=None, src: int = 0, chunk: int = 64, before_reuse=None):
    """Frames ingested ONCE (on rank `src`, from host memory) and broadcast to every rank over
    the backend (RCCL over xGMI: the PCIe link of one GPU carries each frame once; gloo on the
    host in the CPU tests) -- SURVEY §8(e)'s frame distribution for the demo loop
    grid_demo1.py:76-87.  Rank `src` passes (F,H,W) u16 depth, (F,H,W,3) u8 colour and (F,4,4)
    world_to_cam; the others pass None.  Yields (depth, colour, world_to_cam) chunks of up to
    `chunk` frames on every rank: device tensors under RCCL, numpy arrays under gloo.  Device
    chunks alternate between two buffers: before a buffer is overwritten, `before_reuse()` is
    called so that the consumer can finish the work still reading it (chunk k - 2)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    dev = _device(group)
    meta = [None]
    if rank == src:
        depth = np.ascontiguousarray(depth)
        rgb = np.ascontiguousarray(rgb)
        meta = [(tuple(depth.shape), str(depth.dtype), tuple(rgb.shape), np.ascontiguousarray(Tinv, np.float64))]
    dist.broadcast_object_list(meta, src=src, group=group)
    dshape, ddtype, cshape, T = meta[0]
    F = dshape[0]
    ddt = {"uint16": torch.int16, "int16": torch.int16, "float64": torch.float64}[ddtype]
    bufs = []
    for k, f0 in enumerate(range(0, F, chunk)):
        n = min(chunk, F - f0)
        if len(bufs) < 2:
            bufs.append((torch.empty((chunk,) + dshape[1:], dtype=ddt, device=dev),
                         torch.empty((chunk,) + cshape[1:], dtype=torch.uint8, device=dev)))
        bd, bc = bufs[k % 2]
        d, c = bd[:n], bc[:n]
        if k >= 2 and before_reuse is not None:
            before_reuse()  # chunk k - 2 read this buffer
        if rank == src:
            hd = torch.from_numpy(depth[f0:f0 + n].view(np.int16) if ddtype != "float64" else depth[f0:f0 + n])
            hc = torch.from_numpy(rgb[f0:f0 + n])
            if dev.type == "cuda":
                hd, hc = hd.pin_memory(), hc.pin_memory()
            d.copy_(hd, non_blocking=True)
            c.copy_(hc, non_blocking=True)
        # as bytes: neither RCCL nor gloo reduces int16, and a broadcast only moves bytes
        dist.broadcast(d.view(torch.uint8), src=src, group=group)
        dist.broadcast(c, src=src, group=group)
        if dev.type == "cuda":
            torch.cuda.current_stream().synchronize()
            yield d, c, T[f0:f0 + n]
        else:
            dn = d.numpy().view(np.uint16) if ddtype != "float64" else d.numpy()
            yield dn, c.numpy(), T[f0:f0 + n]


def integrate_broadcast(vol, K, depth=None, rgb=None, Tinv=None, group=None, src: int = 0, chunk: int = 64):
    """Integrate host frames held by rank `src` into every rank's shard: each chunk is broadcast
    (broadcast_frames) and integrated asynchronously from device memory while the next chunk
    travels; returns after this rank's shard holds every frame."""
    import torch.distributed as dist
    dev = _device(group)
    hw = None
    for d, c, T in broadcast_frames(depth, rgb, Tinv, group, src, chunk, before_reuse=vol.sync):
        if dev.type == "cuda":
            hw = tuple(d.shape[1:3])
            from . import _ffi
            dk = _ffi.DEPTH_F64_M if d.element_size() == 8 else _ffi.DEPTH_U16_MM
            vol.integrate_batch(d.data_ptr(), c.data_ptr(), K, T, hw=hw, device_ptrs=True, sync=False,
                                depth_kind=dk)
        else:
            vol.integrate_batch(d, c, K, T, sync=False)
    vol.sync()
    dist.barrier(group=group)
