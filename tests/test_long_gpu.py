"""Long runs and the per-rank workloads of BASELINE's 8-GPU configs, on one GPU:

  * config[3] per rank: cyclic column shard 3 of 8 of the 512^3 @ 2 cm volume over 1000 frames
    of the bench trajectory, bit-exact against the oracle on rows of the shard; and over 5000
    frames, where weights cross the LDS reciprocal table's limit by accumulation;
  * the fast-path boundaries: weights around the 4063 limit of the LDS part of the reciprocal
    table and the 65503 limit of the whole table (kRcpTab / kRcpBig less kMaxBatch + 1 = 33 with
    32-frame launches, csrc/tsdf_device.h; the preloaded ranges also straddle the 4079 / 65519 and
    4087 / 65527 of -DTSDF_MAX_BATCH=16 and 8) and non-canonical colours, preloaded with set_state;
  * config[4] per rank: bucket-range hash shard 5 of 8 over a 1024^3 @ 1 cm extent over its whole
    10,000-frame sequence in one asynchronous call (the table doubles under the 0.75 policy and
    the pool grows mid-run), against dense slabs (and those against the oracle) on rows restricted
    to the shard's blocks;
  * the hash's f32 state against the reference's float64 Voxel (voxel.py:19-49) over 500 frames,
    within north_star's 1e-4.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
ROOM = 10.24


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def _frames_on_device(n, start=0, ring=None):
    """n bench-trajectory frames rendered straight into HBM (u16 bits as int16, RGB8)."""
    import torch
    from tsdf_amd import scene
    ring = scene.BENCH_RING if ring is None else ring
    poses = scene.trajectory(n, seed=0, start=start, radius_frac=ring)
    spheres = scene.make_spheres(0, ring_frac=ring)
    dev = torch.device("cuda", 0)
    depth = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((n, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, n, 50):
        d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=start + s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    torch.cuda.synchronize()
    return depth, rgb, poses


def test_config3_rank_shard_1000_frames_matches_oracle_rows():
    """One rank of config[3]: the cyclic column shard 3 of 8 of 512^3 @ 2 cm integrates 1000
    frames (32 batches of up to 32 frames through the pipelined launches); rows at both ends of one of its columns
    and inside two others equal the oracle bit for bit at the end (weights reach the hundreds)."""
    from tsdf_amd import grid_fusion, scene, sharding
    n = 1000
    depth, rgb, poses = _frames_on_device(n)
    K = scene.intrinsics()
    Tinv = np.linalg.inv(poses)
    bnds = np.array([[0.0, ROOM]] * 3)
    vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(3, 8))
    vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=False)
    vol.sync()
    xi = sharding.columns(3, 8, 512)
    rows = np.array([24, 31, 227, 412], np.int64)  # columns 3, 28, 51 (c % 16 in {3, 12})
    assert np.isin(rows, xi).all()
    orc = O.OracleTSDFVolume(bnds.copy(), 0.02, x_index=rows)
    dh = depth.cpu().numpy().view(np.uint16)
    ch = rgb.cpu().numpy()
    n_upd = 0
    for f in range(n):
        n_upd += orc.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[f])
    assert n_upd > 10_000_000
    lr = np.searchsorted(xi, rows)
    t, w, c = vol.get_rows(lr)
    assert _same(t, orc._tsdf_vol_cpu) and _same(w, orc._weight_vol_cpu) and _same(c, orc._color_vol_cpu)
    assert w.max() >= 500 and vol.stats()["list_errors"] == 0


@pytest.fixture(scope="module")
def bench10k():
    """The bench trajectory's first 10,000 frames in HBM (15 GB: u16 depth bits as int16, RGB8),
    shared by the 10k-frame tests of config[3] and config[4]."""
    import torch
    from tsdf_amd import scene
    n = 10000
    dev = torch.device("cuda", 0)
    poses = scene.trajectory(n, seed=0, radius_frac=scene.BENCH_RING)
    spheres = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((n, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, n, 50):
        d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    torch.cuda.synchronize()
    yield depth, rgb, poses
    del depth, rgb
    torch.cuda.empty_cache()


@pytest.mark.timeout(400)
def test_config3_rank_shard_10000_frames_full_sequence(bench10k):
    """config[3]'s whole sequence on one rank (BASELINE: 10k frames; the demo loop is
    grid_demo1.py:76-87): cyclic column shard 3 of 8 of 512^3 @ 2 cm integrates 10,000 frames of
    the bench trajectory (313 32-frame batches through the pipelined launches).  Weights pass the 4063
    limit of the LDS part of the reciprocal table by accumulation alone (no preload), so waves
    move to the HBM table mid-run, and stay below the whole table's 65519.  The two rows holding
    the largest weights equal the oracle bit for bit; the frames stay in HBM (15 GB) and reach
    the host in chunks for the oracle."""
    from tsdf_amd import grid_fusion, scene, sharding
    depth, rgb, poses = bench10k
    n, chunk = len(poses), 1000
    K = scene.intrinsics()
    Tinv = np.linalg.inv(poses)
    bnds = np.array([[0.0, ROOM]] * 3)
    vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(3, 8))
    vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=False)
    vol.sync()
    xi = sharding.columns(3, 8, 512)
    _, W, _ = vol.get_state()
    row_max = W.reshape(len(xi), -1).max(1)
    assert 4087 < row_max.max() < 65519
    pick = np.argsort(row_max)[-2:]  # the two rows with the largest weights
    rows = xi[np.sort(pick)]
    del W
    orc = O.OracleTSDFVolume(bnds.copy(), 0.02, x_index=rows)
    for c0 in range(0, n, chunk):
        dh = depth[c0:c0 + chunk].cpu().numpy().view(np.uint16)
        ch = rgb[c0:c0 + chunk].cpu().numpy()
        for f in range(len(dh)):
            orc.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[c0 + f])
    t, w, c = vol.get_rows(np.searchsorted(xi, rows))
    assert _same(t, orc._tsdf_vol_cpu) and _same(w, orc._weight_vol_cpu) and _same(c, orc._color_vol_cpu)
    assert (w > 4087).sum() > 100 and vol.stats()["list_errors"] == 0
    assert vol.stats()["frames"] == n


@pytest.mark.parametrize("batched,w_lo,limit", [(False, 4050, 4079), (True, 4050, 4079),
                                                (True, 65490, 65519)])
def test_weights_across_the_reciprocal_table_limit_and_odd_colours(batched, w_lo, limit):
    """Preloaded weights around a limit of the RN(1/n) table (its LDS part covers integer weights
    below 4063, then waves read the HBM part; past 65503 the quotients switch to IEEE division;
    the preloads straddle those of 16- and 8-frame builds too)
    and colours that are not the canonical B*65536+G*256+R integers (non-integral, negative,
    >= 2^24), next to canonical ones: every path of the update equals the oracle bit for bit."""
    from tsdf_amd import grid_fusion, scene
    n = 12
    depth, rgb, poses = _frames_on_device(n, start=120, ring=0.34)
    dh, ch = depth.cpu().numpy().view(np.uint16), rgb.cpu().numpy()
    K = scene.intrinsics()
    bnds = np.array([[0.0, ROOM]] * 3)
    vol = grid_fusion.TSDFVolume(bnds.copy(), 0.08)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    shape = tuple(int(x) for x in vol._vol_dim)
    rng = np.random.default_rng(11)
    w0 = rng.integers(w_lo, w_lo + 50, size=shape).astype(np.float32)
    w0[rng.random(shape) < 0.3] = 0.0
    t0 = rng.uniform(-1, 1, size=shape).astype(np.float32)
    canon = (rng.integers(0, 256, size=shape) * 65536 + rng.integers(0, 256, size=shape) * 256
             + rng.integers(0, 256, size=shape)).astype(np.float32)
    odd = rng.choice(np.array([0.5, -3.0, 16777216.0 + 512.0, 123456.75], np.float32), size=shape)
    c0 = np.where(rng.random(shape) < 0.25, odd, canon).astype(np.float32)
    vol.set_state(t0, w0, c0)
    orc._tsdf_vol_cpu[:], orc._weight_vol_cpu[:], orc._color_vol_cpu[:] = t0, w0, c0
    for f in range(n):
        orc.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[f])
    if batched:
        vol.integrate_batch(dh, ch, K, np.linalg.inv(poses))
    else:
        for f in range(n):
            vol.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[f])
    T, W, C = vol.get_state()
    assert (W > limit).any() and (W[W > 0] < limit).any()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)


@pytest.mark.timeout(400)
def test_config4_rank_hash_shard_1024_extent_10000_frames(bench10k):
    """config[4]'s whole per-rank sequence (BASELINE: 10k frames, bucket-range sharded, 1024^3 @
    1 cm; the reference loop is hash_demo1.py:114-125): shard 5 of 8 of a table created with 2^17
    slots (so the reference's 0.75 load-factor policy doubles it mid-run) and a pool of 2^14 blocks
    (grown ahead of the launches in flight), integrating 10,000 bench frames in one asynchronous
    call.  No brick is lost (the fresh table's first batch runs synchronously: the bricks its cull
    found no room for are re-run exactly after the pool grows; every later, asynchronous launch
    finds room, else sync() raises), the table doubled, and on two x rows a voxel is found iff its
    block's home bucket (in the table size of create) is in the shard's range and the dense grid
    updated it, with the dense grid's exact values; the dense rows equal the oracle bit for bit."""
    from tsdf_amd import grid_fusion, hash_fusion, scene, sharding
    depth, rgb, poses = bench10k
    n, chunk = len(poses), 1000
    K = scene.intrinsics()
    Tinv = np.linalg.inv(poses)
    bnds = np.array([[0.0, ROOM]] * 3)
    ht = hash_fusion.HashTable(bnds.copy(), 0.01, 1 << 17, shard=5, n_shards=8, max_blocks=1 << 14)
    assert tuple(int(x) for x in ht._vol_dim) == (1024, 1024, 1024)
    ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=False)
    ht.sync()  # (raises TSDF_E_CAPACITY if an asynchronous launch skipped a brick)
    info = ht.info()
    assert ht.stats()["list_errors"] == 0
    assert info["capacity"] > 1 << 17 and info["used"] > 100_000 and info["pool_capacity"] > 1 << 14
    rows = [300, 700]
    orc = O.OracleTSDFVolume(bnds.copy(), 0.01, x_index=np.array(rows))
    slabs = [grid_fusion.TSDFVolume(bnds.copy(), 0.01, slab=(x, x + 1)) for x in rows]
    for sl in slabs:
        sl.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=False)
    for c0 in range(0, n, chunk):
        dh = depth[c0:c0 + chunk].cpu().numpy().view(np.uint16)
        ch = rgb[c0:c0 + chunk].cpu().numpy()
        for f in range(len(dh)):
            orc.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[c0 + f])
    yy, zz = np.meshgrid(np.arange(1024), np.arange(1024), indexing="ij")
    n_found = n_upd = 0
    for i, (x, sl) in enumerate(zip(rows, slabs)):
        T, W, C = (a[0] for a in sl.get_state())
        assert _same(T, orc._tsdf_vol_cpu[i]) and _same(W, orc._weight_vol_cpu[i]) and _same(C, orc._color_vol_cpu[i])
        own = sharding.hash_owner(x // 8, yy // 8, zz // 8, 1 << 17, 8) == 5
        ijk = np.stack([np.full(yy.size, x), yy.reshape(-1), zz.reshape(-1)], 1)
        found, t, w, c = ht.lookup(ijk)
        found = found.reshape(1024, 1024)
        assert np.array_equal(found, own & (W > 0))
        n_found += int(found.sum())
        n_upd += int((W > 0).sum())
        m = found.reshape(-1)
        assert _same(t[m], T.reshape(-1)[m]) and _same(w[m], W.reshape(-1)[m]) and _same(c[m], C.reshape(-1)[m])
    assert 0 < n_found < n_upd


def test_hash_f32_state_within_1e4_of_reference_f64_voxels_over_500_frames():
    """HashTable.integrate keeps the reference's Voxel in float64 (voxel.py:19-49); the GPU hash
    keeps f32 like the grid.  Over 500 frames the voxel set, weights and colours stay equal and
    tsdf within north_star's 1e-4."""
    from tsdf_amd import hash_fusion, scene
    n = 500
    depth, rgb, poses = _frames_on_device(n, start=0, ring=0.34)
    K = scene.intrinsics()
    bnds = np.array([[0.0, ROOM]] * 3)
    ht = hash_fusion.HashTable(bnds.copy(), 0.08, 1 << 16)
    ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, np.linalg.inv(poses), hw=(480, 640), device_ptrs=True)
    hv = O.OracleHashVolume(bnds.copy(), 0.08)
    dh, ch = depth.cpu().numpy().view(np.uint16), rgb.cpu().numpy()
    for f in range(n):
        hv.integrate(ch[f], dh[f].astype(float) / 1000.0, K, poses[f])
    T, W, C = ht.get_state()
    assert np.array_equal(W > 0, hv.weight > 0)
    assert np.array_equal(W.astype(np.float64), hv.weight) and np.array_equal(C.astype(np.float64), hv.color)
    drift = np.abs(T.astype(np.float64) - hv.sdf).max()
    assert hv.weight.max() >= 400
    assert drift <= 1e-4, drift
