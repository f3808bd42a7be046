"""The multi-GPU end of the path through the HIP library (BASELINE config[3] / config[4] per
rank): shards on one GPU, meshed with their neighbours' border rows, gathered and merged --
equal to one unsharded volume.  The single-process tests assemble the halos directly; the
world_size-2 test runs tests/dist_gpu_worker.py under torch.distributed (gloo: both ranks share
the box's one GPU) and exercises the point-to-point exchange, the gather and the sparse hash
merge of tsdf_amd.sharding."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, load_lounge, lounge_intrinsics

pytestmark = pytest.mark.gpu
C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]


def _integrated(vols, n=3):
    K = lounge_intrinsics()
    for f in range(n):
        _, depth, rgb, pose = load_lounge(f)
        for v in vols:
            v.integrate(rgb, depth, K, pose)


def _halo_from(parts, p):
    """The border rows part p needs, read from the parts that own them."""
    need = p.mesh_halo_rows()
    if len(need) == 0:
        return None
    owner = {}
    for q in parts:
        for lr, g in enumerate(q.x_index):
            owner[int(g)] = (q, lr)
    ts, cs = [], []
    for g in need:
        q, lr = owner[int(g)]
        t, _, c = q.get_rows([lr], weight=False)
        ts.append(t[0])
        cs.append(c[0])
    return need, np.stack(ts), np.stack(cs)


def _sorted_faces(v_keys, faces):
    k = v_keys[faces]
    return k[np.lexsort(k.T[::-1])]


@pytest.mark.parametrize("layout,world", [("cyclic", 2), ("cyclic", 3), ("cyclic", 8), ("slab", 3)])
def test_shard_meshes_unite_to_the_unsharded_mesh(layout, world):
    """Union of N shard meshes (each with its halo) == the unsharded mesh: vertices, normals and
    colours bit-identical in the same (voxel, axis) order, the same set of triangles."""
    from tsdf_amd import _ffi, grid_fusion, sharding
    bnds = np.array([[-2.56, 1.48], [-2.56, 2.56], [0.0, 5.12]])  # X = 101: a ragged last column
    full = grid_fusion.TSDFVolume(bnds.copy(), 0.04)
    X = int(full._vol_dim[0])
    if layout == "cyclic":
        parts = [grid_fusion.TSDFVolume(bnds.copy(), 0.04, shard=(r, world)) for r in range(world)]
    else:
        parts = [grid_fusion.TSDFVolume(bnds.copy(), 0.04, slab=sharding.slab(r, world, X)) for r in range(world)]
    _integrated([full] + parts)
    v, n, c, f, k = full.extract_mesh(keys=True)
    assert len(f) > 5000 and np.all(np.diff(k) > 0)
    meshes = []
    for p in parts:
        halo = _halo_from(parts, p)
        pv, pn, pc, pf, pk = p.extract_mesh(halo=halo, global_x=X, keys=True)
        meshes.append((pv, pf, pn, pc, pk))
    mv, mf, mn, mc = sharding.merge_meshes(meshes)
    assert np.array_equal(mv.view(np.uint32), v.view(np.uint32))
    assert np.array_equal(mn.view(np.uint32), n.view(np.uint32)) and np.array_equal(mc, c)
    uk = np.unique(np.concatenate([m[4] for m in meshes]))
    assert np.array_equal(uk, k)
    assert np.array_equal(_sorted_faces(k, mf), _sorted_faces(k, f))
    assert sum(len(m[1]) for m in meshes) == len(f)  # every cell owned by exactly one shard
    if layout == "cyclic":
        gappy = max(parts, key=lambda p: len(p.x_index))  # (at X = 101, shard 0 of 8 holds one column)
        with pytest.raises(_ffi.TSDFError):
            gappy.extract_mesh()  # a cyclic shard alone would mesh across its column gaps


def test_slab_alone_meshes_its_sub_volume_in_world_coordinates():
    """A slab meshed without halo is the mesh of its own sub-volume at world positions: every
    vertex has the global key, position and colour of the unsharded mesh's vertex on the same
    edge, and its triangles are the unsharded mesh's cells inside the slab."""
    from tsdf_amd import grid_fusion
    full = grid_fusion.TSDFVolume(np.array(C1), 0.04)
    sl = grid_fusion.TSDFVolume(np.array(C1), 0.04, slab=(40, 90))
    _integrated([full, sl])
    v, n, c, f, k = full.extract_mesh(keys=True)
    sv, sn, sc, sf, sk = sl.extract_mesh(keys=True)
    idx = np.searchsorted(k, sk)
    assert np.array_equal(k[idx], sk)
    assert np.array_equal(sv.view(np.uint32), v[idx].view(np.uint32)) and np.array_equal(sc, c[idx])
    full_faces = set(map(tuple, k[f].tolist()))
    slab_faces = set(map(tuple, k[idx[sf]].tolist()))
    assert slab_faces <= full_faces  # same triangles, same orientation
    gx = (k[f] // 3) // (128 * 128)  # x of each face's vertices
    deep = (gx.min(1) >= 41) & (gx.max(1) <= 88)  # cells well inside the slab
    assert set(map(tuple, k[f[deep]].tolist())) <= slab_faces and len(sf) > deep.sum() > 1000


def test_rows_and_block_export_round_trip():
    """tsdf_dense_get_rows (any row list) equals get_state's rows; a hash table's exported blocks
    imported into a fresh table reproduce its state and entries."""
    from tsdf_amd import grid_fusion, hash_fusion
    vol = grid_fusion.TSDFVolume(np.array(C1), 0.04)
    ht = hash_fusion.HashTable(np.array(C1), 0.04, 1 << 14)
    _integrated([vol, ht], 2)
    T, W, C = vol.get_state()
    rows = [5, 77, 3, 127]
    t, w, c = vol.get_rows(rows)
    assert np.array_equal(t, T[rows]) and np.array_equal(w, W[rows]) and np.array_equal(c, C[rows])
    ht.add_entries([[1, 2, 3]], tsdf=[0.5], weight=[0.0], color=[7.0])  # weight-0 entry survives
    blocks = ht.export_blocks()
    fresh = hash_fusion.HashTable(np.array(C1), 0.04, 64, max_blocks=64)
    fresh.import_blocks(*blocks)
    for a, b in zip(ht.get_state(), fresh.get_state()):
        assert np.array_equal(a, b)
    assert fresh.count_num_hash_entries() == ht.count_num_hash_entries()
    assert fresh.lookup([[1, 2, 3]])[0][0]


def test_device_buffers_equal_the_host_path():
    """The entry points the RCCL branches of sharding.py call, single-process, with CUDA tensors:
    get_rows(out=<cuda>), extract_mesh(halo=<cuda>) through TSDF_DEVICE_PTRS, and
    export_blocks(device=) -> import_blocks(<cuda>) including non-contiguous tensors -- each
    bit-equal to the host-array path."""
    import torch
    from tsdf_amd import grid_fusion, hash_fusion
    bnds = np.array([[-2.56, 1.48], [-2.56, 2.56], [0.0, 5.12]])
    X = 101
    parts = [grid_fusion.TSDFVolume(bnds.copy(), 0.04, shard=(r, 3)) for r in range(3)]
    ht = hash_fusion.HashTable(bnds.copy(), 0.04, 1 << 14)
    _integrated(parts + [ht], 3)
    p = parts[1]
    # rows into device buffers
    rows = np.array([0, len(p.x_index) - 1, 3], np.int64)
    Y, Z = int(p._local_dim[1]), int(p._local_dim[2])
    out = [torch.full((3, Y, Z), -7.0, device="cuda"), None, torch.full((3, Y, Z), -7.0, device="cuda")]
    p.get_rows(rows, out=out)
    torch.cuda.synchronize()
    t, _, c = p.get_rows(rows, weight=False)
    assert np.array_equal(out[0].cpu().numpy().view(np.uint32), t.view(np.uint32))
    assert np.array_equal(out[2].cpu().numpy().view(np.uint32), c.view(np.uint32))
    # a halo in device memory meshes exactly as the host halo
    gx, ht_h, hc_h = _halo_from(parts, p)
    host = p.extract_mesh(halo=(gx, ht_h, hc_h), global_x=X, keys=True)
    dev_t, dev_c = torch.from_numpy(ht_h).cuda(), torch.from_numpy(hc_h).cuda()
    torch.cuda.synchronize()
    devm = p.extract_mesh(halo=(gx, dev_t, dev_c), global_x=X, keys=True)
    for a, b in zip(host, devm):
        assert np.array_equal(a, b)
    assert len(host[3]) > 1000
    # sparse blocks through device tensors, contiguous and not
    blocks = ht.export_blocks(device="cuda")
    host_blocks = ht.export_blocks()
    dev_np = [x.cpu().numpy() for x in blocks]
    oa = np.lexsort(dev_np[0].T[::-1])  # (the export order follows the table walk: compare by block)
    ob = np.lexsort(host_blocks[0].T[::-1])
    for a, b in zip(dev_np, host_blocks):
        assert np.array_equal(a[oa].view(np.uint32 if a.dtype != np.int64 else np.uint64),
                              b[ob].view(np.uint32 if b.dtype != np.uint64 else np.uint64))
    fresh = hash_fusion.HashTable(bnds.copy(), 0.04, 64, max_blocks=64)
    fresh.import_blocks(*blocks)
    strided = [b.t().contiguous().t() if b.dim() == 2 else b for b in blocks]  # column-major views
    assert not strided[1].is_contiguous()
    fresh2 = hash_fusion.HashTable(bnds.copy(), 0.04, 64, max_blocks=64)
    fresh2.import_blocks(*strided)
    for a, b, c2 in zip(ht.get_state(), fresh.get_state(), fresh2.get_state()):
        assert np.array_equal(a, b) and np.array_equal(a, c2)
    assert fresh2.count_num_hash_entries() == ht.count_num_hash_entries()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("buffers", ["host", "cuda"])
def test_two_rank_job_exchange_gather_and_hash_merge(tmp_path, buffers):
    """buffers="cuda": gather_volume reads rows into device tensors, exchange_halo hands device
    halos to the library, merge_hash_shards exports / imports device blocks, integrate_broadcast
    integrates broadcast device chunks -- the RCCL branches of sharding.py, moved by gloo."""
    from tsdf_amd import grid_fusion, hash_fusion
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(REPO, "tests", "dist_gpu_worker.py"), str(tmp_path), buffers]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    g = np.load(os.path.join(tmp_path, "dist.npz"))
    full = grid_fusion.TSDFVolume(np.array(C1), 0.04)
    hfull = hash_fusion.HashTable(np.array(C1), 0.04, 1 << 16)
    _integrated([full, hfull])
    v, n, c, f, k = full.extract_mesh(keys=True)
    assert np.array_equal(g["v"].view(np.uint32), v.view(np.uint32)) and np.array_equal(g["c"], c)
    assert np.array_equal(_sorted_faces(k, g["f"]), _sorted_faces(k, f))
    assert 0 < int(g["part_verts"]) < len(v)
    T, W, C = full.get_state()
    assert np.array_equal(g["t"], T) and np.array_equal(g["w"], W) and np.array_equal(g["col"], C)
    for a, b in zip((g["ht"], g["hw"], g["hc"]), hfull.get_state()):
        assert np.array_equal(a, b)
    assert int(g["merged_used"]) == int(g["shard_blocks"]) == hfull.info()["used"]
    assert int(g["bcast_ok"]) == 2  # both ranks: broadcast-fed shard == host-fed shard
    assert int(g["dev"]) == (buffers == "cuda")
