"""The N>1 path on the CPU: world_size-2 `gloo` jobs that partition the volume exactly as the GPU
ranks do (tsdf_amd.sharding), integrate each shard with the oracle, and gather/merge the shards.
The result must equal one unsharded oracle volume bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_lounge, lounge_intrinsics

C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _dense_worker(rank, world, port, out_dir, cyclic=False):
    import oracle as O
    from tsdf_amd import sharding
    dist = _init(rank, world, port)
    nx = int(O.OracleTSDFVolume(np.array(C1), 0.04)._vol_dim[0])
    if cyclic:
        xi = sharding.columns(rank, world, nx)
        vol = O.OracleTSDFVolume(np.array(C1), 0.04, x_index=xi)
    else:
        x0, x1 = sharding.slab(rank, world, nx)
        xi = np.arange(x0, x1)
        vol = O.OracleTSDFVolume(np.array(C1), 0.04, slab=(x0, x1))
    K = lounge_intrinsics()
    n = 0
    for f in range(2):
        _, depth, rgb, pose = load_lounge(f)
        n += vol.integrate(rgb, depth, K, pose)
    full = [sharding.gather_rows(a, xi, nx)
            for a in (vol._tsdf_vol_cpu, vol._weight_vol_cpu, vol._color_vol_cpu)]
    tot = sharding.sum_counters({"updates": n})
    if rank == 0:
        np.savez(os.path.join(out_dir, f"dense{int(cyclic)}.npz"), t=full[0], w=full[1], c=full[2], n=tot["updates"])
    dist.destroy_process_group()


def _hash_worker(rank, world, port, out_dir):
    import oracle as O
    from tsdf_amd import sharding
    dist = _init(rank, world, port)
    hv = O.OracleHashVolume(np.array(C1), 0.04)
    K = lounge_intrinsics()
    _, depth, rgb, pose = load_lounge(0)
    hv.integrate(rgb, depth, K, pose)
    # keep only the blocks this rank owns (bucket-range ownership over a 2^16-slot table)
    X, Y, Z = (int(d) for d in hv._vol_dim)
    bx, by, bz = np.meshgrid(np.arange(X) // 8, np.arange(Y) // 8, np.arange(Z) // 8, indexing="ij")
    own = sharding.hash_owner(bx, by, bz, 1 << 16, world) == rank
    t = np.where(own, hv.sdf, 1.0).astype(np.float32)
    w = np.where(own, hv.weight, 0.0).astype(np.float32)
    c = np.where(own, hv.color, 0.0).astype(np.float32)
    T, W, C = sharding.merge_hash_exports(t, w, c)
    if rank == 0:
        np.savez(os.path.join(out_dir, "hash.npz"), t=T, w=W, c=C, owned=int(own.sum()))
    dist.destroy_process_group()


class _FakeShard:
    """Host stand-in for a sharded TSDFVolume (the attributes and calls tsdf_amd.sharding uses),
    backed by an oracle volume's arrays: lets the exchange / gather logic run under gloo on the
    CPU.  mesh_halo_rows restates csrc/tsdf_mesh.hip mesh_halo_rows."""

    def __init__(self, full, x_index):
        self.x_index = np.asarray(x_index, np.int64)
        self._vol_dim = np.array(full[0].shape, np.int64)
        self._local_dim = np.array([len(self.x_index)] + list(full[0].shape[1:]), np.int64)
        self._rows = [a[self.x_index] for a in full]

    def mesh_halo_rows(self, global_x=None):
        X = int(global_x or self._vol_dim[0])
        local = np.zeros(X, bool)
        local[self.x_index] = True
        need = set()
        for g in self.x_index:
            need |= {g - 1, g + 1} | ({g + 2} if g + 1 < X and not local[g + 1] else set())
        return np.array(sorted(g for g in need if 0 <= g < X and not local[g]), np.int64)

    def get_rows(self, local_rows, weight=True, out=None):
        lr = np.asarray(local_rows, np.int64)
        t, w, c = (a[lr] for a in self._rows)
        return t, (w if weight else None), c


def _halo_worker(rank, world, port, out_dir):
    import oracle as O
    from tsdf_amd import sharding
    dist = _init(rank, world, port)
    full = O.OracleTSDFVolume(np.array(C1), 0.04)
    _, depth, rgb, pose = load_lounge(0)
    full.integrate(rgb, depth, lounge_intrinsics(), pose)
    arrs = (full._tsdf_vol_cpu, full._weight_vol_cpu, full._color_vol_cpu)
    X = arrs[0].shape[0]
    sh = _FakeShard(arrs, sharding.columns(rank, world, X))
    gx, ht, hc = sharding.exchange_halo(sh)
    ok = bool(np.array_equal(gx, sh.mesh_halo_rows()) and np.array_equal(ht, arrs[0][gx])
              and np.array_equal(hc, arrs[2][gx]))
    oks = [None] * world
    dist.all_gather_object(oks, ok)
    state = sharding.gather_volume(sh)
    if rank == 0:
        np.savez(os.path.join(out_dir, "halo.npz"), ok=np.array(oks), t=state[0], w=state[1], c=state[2],
                 n_halo=len(gx))
    dist.destroy_process_group()


def _broadcast_worker(rank, world, port, out_dir):
    """Rank 0 alone reads the lounge frames; every rank receives them by broadcast and integrates
    its cyclic shard with the oracle; the gathered volume must be the unsharded one."""
    import oracle as O
    from tsdf_amd import sharding
    dist = _init(rank, world, port)
    nx = int(O.OracleTSDFVolume(np.array(C1), 0.04)._vol_dim[0])
    xi = sharding.columns(rank, world, nx)
    vol = O.OracleTSDFVolume(np.array(C1), 0.04, x_index=xi)
    K = lounge_intrinsics()
    d = c = T = None
    if rank == 0:
        fr = [load_lounge(f) for f in range(3)]
        d = np.stack([f[0] for f in fr]).astype(np.uint16)
        c = np.stack([f[2] for f in fr])
        T = np.linalg.inv(np.stack([f[3] for f in fr]))
    got = 0
    for dd, cc, tt in sharding.broadcast_frames(d, c, T, chunk=2):
        for i in range(len(dd)):
            m = dd[i].astype(float) / 1000.0
            m[m == 65.535] = 0
            vol.integrate(cc[i], m, K, np.linalg.inv(tt[i]))
            got += 1
    full = [sharding.gather_rows(a, xi, nx) for a in (vol._tsdf_vol_cpu, vol._weight_vol_cpu, vol._color_vol_cpu)]
    if rank == 0:
        np.savez(os.path.join(out_dir, "bcast.npz"), t=full[0], w=full[1], c=full[2], got=got)
    dist.destroy_process_group()


def _cyclic_worker(rank, world, port, out_dir):
    _dense_worker(rank, world, port, out_dir, cyclic=True)


def _run(fn, tmp_path, world=2):
    mp.start_processes(fn, args=(world, _port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")


def test_slab_partition_properties():
    from tsdf_amd import sharding
    for nx in (1, 7, 8, 100, 128, 405, 512, 1024):
        for world in (1, 2, 3, 4, 8):
            parts = [sharding.slab(r, world, nx) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == nx
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            if nx >= 8 * world:
                assert all(p[0] % 8 == 0 for p in parts)
                assert all(p[1] > p[0] for p in parts)


def test_cyclic_columns_partition():
    from tsdf_amd import sharding
    for nx in (16, 101, 128, 512, 1000):
        for world in (1, 2, 3, 8):
            if -(-nx // 8) < world:
                continue
            cols = [sharding.columns(r, world, nx) for r in range(world)]
            allx = np.sort(np.concatenate(cols))
            assert np.array_equal(allx, np.arange(nx))
            assert max(len(c) for c in cols) - min(len(c) for c in cols) <= 8
            assert all((np.diff(c) > 0).all() for c in cols)  # local rows in global x order


def test_cyclic_columns_mirrored_pairs_even_out_an_x_ramp():
    """Shard s owns columns s and 2N-1-s of every 2N (tsdf_dense_create_shard): a work density
    linear in x gives every rank the same total over whole periods (plain c % N == s gave rank
    0 the lightest column of every period)."""
    from tsdf_amd import sharding
    for world in (2, 4, 8):
        nx = 512
        tot = [sharding.columns(r, world, nx).sum() for r in range(world)]
        assert len(set(tot)) == 1
        assert list(sharding.columns(1, world, nx)[8:16] // 8) == [2 * world - 2] * 8


def test_hash_owner_matches_oracle_keys():
    import oracle as O
    from tsdf_amd import sharding
    rng = np.random.default_rng(3)
    b = rng.integers(0, 128, size=(500, 3))
    for bits in (64, 32):
        home = O.hash_keys(b, 1 << 22, bits)
        assert np.array_equal(sharding.ref_hash(b[:, 0], b[:, 1], b[:, 2], 1 << 22, bits), home)
        assert np.array_equal(sharding.hash_owner(b[:, 0], b[:, 1], b[:, 2], 1 << 22, 8, bits), home * 8 // (1 << 22))


@pytest.mark.parametrize("cyclic", [False, True])
def test_dense_slabs_two_ranks_gloo(tmp_path, cyclic):
    import oracle as O
    _run(_cyclic_worker if cyclic else _dense_worker, tmp_path)
    g = np.load(os.path.join(tmp_path, f"dense{int(cyclic)}.npz"))
    ref = O.OracleTSDFVolume(np.array(C1), 0.04)
    K = lounge_intrinsics()
    n = 0
    for f in range(2):
        _, depth, rgb, pose = load_lounge(f)
        n += ref.integrate(rgb, depth, K, pose)
    assert np.array_equal(g["t"].view(np.uint32), ref._tsdf_vol_cpu.view(np.uint32))
    assert np.array_equal(g["w"], ref._weight_vol_cpu) and np.array_equal(g["c"], ref._color_vol_cpu)
    assert int(g["n"]) == n


def test_hash_bucket_ranges_two_ranks_gloo(tmp_path):
    import oracle as O
    _run(_hash_worker, tmp_path)
    g = np.load(os.path.join(tmp_path, "hash.npz"))
    hv = O.OracleHashVolume(np.array(C1), 0.04)
    _, depth, rgb, pose = load_lounge(0)
    hv.integrate(rgb, depth, lounge_intrinsics(), pose)
    assert np.array_equal(g["w"], hv.weight.astype(np.float32))
    assert np.array_equal(g["c"], hv.color.astype(np.float32))
    assert np.array_equal(g["t"], hv.sdf.astype(np.float32))
    assert 0 < int(g["owned"]) < hv.weight.size


@pytest.mark.parametrize("world", [2, 3])
def test_halo_exchange_and_device_gather_logic_gloo(tmp_path, world):
    """sharding.exchange_halo (every rank's border rows for sharded marching cubes, traded point
    to point) and sharding.gather_volume on world_size 2 and 3 over gloo: each rank receives
    exactly the rows mesh_halo_rows asks for, with the owners' values, and rank 0 reassembles the
    whole volume."""
    import oracle as O
    mp.start_processes(_halo_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    g = np.load(os.path.join(tmp_path, "halo.npz"))
    assert g["ok"].all() and int(g["n_halo"]) > 0
    full = O.OracleTSDFVolume(np.array(C1), 0.04)
    _, depth, rgb, pose = load_lounge(0)
    full.integrate(rgb, depth, lounge_intrinsics(), pose)
    assert np.array_equal(g["t"], full._tsdf_vol_cpu) and np.array_equal(g["w"], full._weight_vol_cpu)
    assert np.array_equal(g["c"], full._color_vol_cpu)


def test_merge_meshes_unites_by_key():
    """merge_meshes: duplicated border vertices collapse to one, ordered by key; faces follow."""
    from tsdf_amd import sharding
    v = np.arange(15, dtype=np.float32).reshape(5, 3)
    a = (v[[0, 1, 2]], np.array([[0, 1, 2]], np.int32), v[[0, 1, 2]], np.zeros((3, 3), np.uint8), np.array([10, 20, 30]))
    b = (v[[2, 3, 4]], np.array([[0, 2, 1]], np.int32), v[[2, 3, 4]], np.ones((3, 3), np.uint8), np.array([30, 5, 40]))
    mv, mf, mn, mc = sharding.merge_meshes([a, b])
    assert np.array_equal(mv, v[[3, 0, 1, 2, 4]])  # keys 5, 10, 20, 30, 40
    assert np.array_equal(mf, np.array([[1, 2, 3], [3, 4, 0]]))


def test_frames_ingested_once_and_broadcast_gloo(tmp_path):
    """SURVEY §8(e) frame distribution: one rank ingests the host frames, the others receive them
    by broadcast in chunks (sharding.broadcast_frames); each rank's shard then equals the same
    rows of the unsharded volume."""
    import oracle as O
    _run(_broadcast_worker, tmp_path)
    g = np.load(os.path.join(tmp_path, "bcast.npz"))
    ref = O.OracleTSDFVolume(np.array(C1), 0.04)
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        ref.integrate(rgb, depth, K, pose)
    assert int(g["got"]) == 3
    assert np.array_equal(g["t"].view(np.uint32), ref._tsdf_vol_cpu.view(np.uint32))
    assert np.array_equal(g["w"], ref._weight_vol_cpu) and np.array_equal(g["c"], ref._color_vol_cpu)
