"""The reference's call pattern through the drop-in wrappers: one integrate() per host frame
(grid_demo1.py:76-87, hash_demo1.py:39), float64 metres as the demos pass them, deferred into
batches of 8 frames on the device (TSDF_DEFER) -- bit-exact against the oracle whatever the
flush points; and the asynchronous hash path's pool growth / overflow reporting.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BNDS = [[0.0, 10.24]] * 3


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def _synth(n, start=0):
    from tsdf_amd import scene
    poses = scene.trajectory(n, seed=0, start=start)
    d, c = scene.render(poses, scene.make_spheres(0), seed=0, start=start)
    return np.ascontiguousarray(d.numpy()), np.ascontiguousarray(c.numpy()), poses


def test_deferred_per_frame_integrate_matches_oracle():
    """19 per-frame calls with f64 metres (half of them not millimetre-exact, so deferred batches
    staged as u16 millimetres are flushed early by a frame that stays f64), varying obs_weight, a
    change of intrinsics mid-stream and reads in between (each read runs the pending frames
    first): deferred, undeferred and the oracle agree bit for bit."""
    from tsdf_amd import grid_fusion
    d, c, poses = _synth(19, start=333)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    K2 = K.copy()
    K2[0, 0] = 590.0
    rng = np.random.default_rng(3)
    dv = grid_fusion.TSDFVolume(np.array(BNDS), 0.08)  # defer=True is the default
    nv = grid_fusion.TSDFVolume(np.array(BNDS), 0.08, defer=False)
    orc = O.OracleTSDFVolume(np.array(BNDS), 0.08)
    n_orc = 0
    for f in range(19):
        m = d[f].astype(float) / 1000.0
        if f % 2:
            m = m + rng.uniform(0, 1e-5, size=m.shape) * (m > 0)
        Kf = K2 if 9 <= f < 12 else K
        ow = 1.0 if f % 5 else 0.5
        for v in (dv, nv):
            v.integrate(c[f], m, Kf, poses[f], obs_weight=ow)
        n_orc += orc.integrate(c[f], m, Kf, poses[f], obs_weight=ow)
        if f in (4, 13):
            T, W, C = dv.get_state()
            assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)
    assert dv.stats()["voxel_updates"] == nv.stats()["voxel_updates"] == n_orc
    for a, b, o in zip(dv.get_state(), nv.get_state(), (orc._tsdf_vol_cpu, orc._weight_vol_cpu, orc._color_vol_cpu)):
        assert _same(a, o) and _same(b, o)


@pytest.mark.parametrize("mm", ["1", "0"])
def test_deferred_millimetre_metres_staged_as_u16(monkeypatch, mm):
    """The demos' depth (png / 1000.: every value RN(k / 1000)) is staged as u16 millimetres by the
    deferred per-frame calls (a quarter of the bytes over PCIe; TSDF_DEFER_MM=0 stages the f64 as
    it comes): 20 frames -- two full deferred batches and a flushed partial one -- equal the oracle
    bit for bit either way, and the hash table equals the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion
    monkeypatch.setenv("TSDF_DEFER_MM", mm)
    d, c, poses = _synth(20, start=470)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    dv = grid_fusion.TSDFVolume(np.array(BNDS), 0.08)
    hv = hash_fusion.HashTable(np.array(BNDS), 0.08)
    orc = O.OracleTSDFVolume(np.array(BNDS), 0.08)
    n = 0
    for f in range(20):
        m = d[f].astype(float) / 1000.0
        dv.integrate(c[f], m, K, poses[f])
        hv.integrate(c[f], m, K, poses[f])
        n += orc.integrate(c[f], m, K, poses[f])
    T, W, C = dv.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)
    assert dv.stats()["voxel_updates"] == n
    for a, b in zip(dv.get_state(), hv.get_state()):  # (the hash equals the dense grid)
        assert np.array_equal(a, b)


def test_deferred_hash_per_frame_matches_dense():
    """HashTable.integrate per frame (deferred: the call that fills a batch launches it, and the
    next call checks it -- a full table / pool grows and the skipped bricks re-run exactly before
    any later frame) equals the dense grid; 29 frames = three such checks by per-frame calls and
    one by the read."""
    from tsdf_amd import grid_fusion, hash_fusion
    d, c, poses = _synth(29, start=610)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.08, defer=False)
    h = hash_fusion.HashTable(np.array(BNDS), 0.08, 37, max_blocks=16)
    for f in range(29):
        m = d[f].astype(float) / 1000.0
        g.integrate(c[f], m, K, poses[f])
        h.integrate(c[f], m, K, poses[f])
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)
    assert h.info()["capacity"] > 37 and h.info()["pool_capacity"] > 16


def test_async_hash_overflow_is_reported_not_replayed(monkeypatch):
    """A pool far too small for asynchronous launches: the skipped bricks cannot be re-run (their
    frames are gone), so the library reports TSDF_E_CAPACITY once, clears the overflow list (no
    later call replays it against other frames), and the handle works again after reset().  (The
    copy-grown pool: a mapped pool grows in 32 MB pieces, which hold this whole extent; and no
    growth ahead of the asynchronous launches, TSDF_HASH_ASYNC_GROW=0, which would otherwise keep
    room for them.)"""
    from tsdf_amd import _ffi, grid_fusion, hash_fusion
    monkeypatch.setenv("TSDF_HASH_VMM", "0")
    monkeypatch.setenv("TSDF_HASH_ASYNC_GROW", "0")
    d, c, poses = _synth(24, start=700)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.08, 1 << 12, max_blocks=64)
    # not a fresh table (whose first asynchronous batch would run synchronously): one synchronous
    # frame that updates nothing
    h.integrate_batch(np.zeros_like(d[:1]), c[:1], K, Tinv[:1])
    with pytest.raises(_ffi.TSDFError) as ei:
        h.integrate_batch(d, c, K, Tinv, sync=False)
        h.sync()
    assert ei.value.code == _ffi.E_CAPACITY and "skipped" in str(ei.value)
    assert h.stats()["bricks_skipped"] > 0
    h.sync()  # reported once
    h.reset()
    h.integrate_batch(d, c, K, Tinv)  # synchronous: grows and re-runs exactly
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.08)
    g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("pipe,vmm", [("1", "1"), ("0", "1"), ("1", "0")])
def test_async_hash_grows_ahead_of_the_pool(monkeypatch, pipe, vmm):
    """Asynchronous hash calls read each launch's pool report two launches later and grow the
    pool / table before they fill: a continuing trajectory needs several growths and none of its
    bricks is skipped; the result equals the dense grid.  The pool grows by mapping memory behind
    its reserved address ranges (vmm = 1, launches in flight keep running) or, with
    TSDF_HASH_VMM=0, by a drained copy into larger allocations."""
    from tsdf_amd import grid_fusion, hash_fusion
    monkeypatch.setenv("TSDF_PIPELINE", pipe)
    monkeypatch.setenv("TSDF_HASH_VMM", vmm)
    # 8-frame launches: eight asynchronous launches after the synchronous start (with 32-frame
    # launches the two left fit the room the start leaves, and nothing would need to grow)
    monkeypatch.setenv("TSDF_BATCH", "8")
    d, c, poses = _synth(72, start=100)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    # 512^3: ~56k blocks by the end, many pool pieces (4096 blocks each) past the first batch's
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 12, max_blocks=256)
    h.integrate_batch(d[:8], c[:8], K, Tinv[:8])  # synchronous start
    cap0 = h.info()["pool_capacity"]
    skipped0 = h.stats()["bricks_skipped"]
    h.integrate_batch(d[8:], c[8:], K, Tinv[8:], sync=False)
    h.sync()
    assert h.stats()["bricks_skipped"] == skipped0
    info = h.info()
    assert info["pool_capacity"] > cap0 and info["capacity"] > 1 << 12
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("max_load", [None, "0.97"])
def test_async_hash_table_grows_before_the_launches_in_flight_fill_it(monkeypatch, max_load):
    """The load-factor sweep's policy run (tools/hash_sweep.py; it skipped bricks in round 4): a
    2^17-slot table, asynchronous calls over the bench ring's 1000 frames.  The table must double
    before the two launches in flight can fill its slots -- under the reference's 0.75 policy
    (growth can jump just below the threshold) and with the policy lifted to 0.97 -- so no brick
    is skipped, and the result equals the dense grid."""
    import torch
    from tsdf_amd import grid_fusion, hash_fusion, scene
    if max_load:
        monkeypatch.setenv("TSDF_HASH_MAX_LOAD", max_load)
    n = 1000
    poses = scene.trajectory(n, seed=0, radius_frac=scene.BENCH_RING)
    sph = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    dev = torch.device("cuda", 0)
    depth = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((n, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, n, 50):
        d, c = scene.render(poses[s:s + 50], sph, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    torch.cuda.synchronize()
    K = scene.intrinsics()
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 17, max_blocks=1 << 15)
    # (a fresh table's first batch runs synchronously -- explicitly here -- and its pool overflow
    # re-runs exactly; bricks_skipped counts those re-run bricks too)
    nb = h.frames_per_launch()
    h.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv[:nb], hw=(480, 640), device_ptrs=True)
    skipped0 = h.stats()["bricks_skipped"]
    h.integrate_batch(depth[nb:].data_ptr(), rgb[nb:].data_ptr(), K, Tinv[nb:], hw=(480, 640), device_ptrs=True,
                      sync=False)
    h.sync()  # (raises TSDF_E_CAPACITY if an asynchronous launch skipped a brick)
    assert h.stats()["bricks_skipped"] == skipped0
    info = h.info()
    assert info["capacity"] > 1 << 17 and info["used"] > 100_000
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    g.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True)
    del depth, rgb
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


def test_deferred_hash_restage_after_a_pending_overflow():
    """Round-2 advisor finding: a per-frame call that fills a batch launches it and leaves its
    overflow check (grow, exact re-run of the skipped bricks) to the next call; that re-run reads
    the batch's staging slots.  A power-of-two table (the fused launch, which defers the check)
    with the smallest pool overflows in the first batch; the next frame is larger, so the staging
    slots are reallocated -- the pending re-run must happen first.  Equal to the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion
    d, c, poses = _synth(12, start=420)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Kh = K.copy()
    Kh[:2] /= 2.0
    Kh[0, 2] -= 0.25  # pixel (u, v) of the half image is pixel (2u + 0.5, 2v + 0.5) of the full one
    Kh[1, 2] -= 0.25
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.08, defer=False)
    h = hash_fusion.HashTable(np.array(BNDS), 0.08, 1 << 6, max_blocks=64)
    for f in range(12):
        half = f < 8  # a full deferred batch of 320x240 frames, then 640x480
        m = (d[f, ::2, ::2] if half else d[f]).astype(float) / 1000.0
        col = np.ascontiguousarray(c[f, ::2, ::2] if half else c[f])
        Kf = Kh if half else K
        g.integrate(col, np.ascontiguousarray(m), Kf, poses[f])
        h.integrate(col, np.ascontiguousarray(m), Kf, poses[f])
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)
    assert h.stats()["bricks_skipped"] > 0  # the deferred overflow re-run did run
    assert h.info()["pool_capacity"] > 64


@pytest.mark.parametrize("map_size", [1000, 1000000, 2000000])
def test_reference_table_sizes_take_the_fused_launch(map_size):
    """HashTable(map_size=10^6) (the reference default, hash_fusion.py:34) and 2*10^6
    (hash_demo1.py:110): the device table is the next power of two, so they run the fused z-half
    launch; hash_function keeps the reference's modulus; results equal the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion
    d, c, poses = _synth(16, start=250)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.04, map_size)
    info = h.info()
    assert info["capacity"] == map_size and info["slots"] == 1 << (map_size - 1).bit_length()
    xyz = np.array([[3, 1000, -7], [123456, 5, 99]], np.int64)
    for p in xyz:
        ref = ((int(p[0]) * 73856093) ^ (int(p[1]) * 19349669) ^ (int(p[2]) * 83492791)) % map_size
        assert h.hash_function(p) == ref
    h.set_profiling(True)
    h.integrate_batch(d, c, K, Tinv)
    st = h.stats()
    assert st["bricks_skipped"] == 0 or map_size == 1000
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.04)
    g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)
    info = h.info()
    assert info["used"] < 0.75 * info["capacity"] + 1 and info["slots"] >= info["capacity"]


def test_f64_device_frames_match_the_u16_encoding():
    """f64-metre frames from device pointers (the drop-in's depth kind on the fused k_fused<DK=1>
    and k_fused_hash<1> launches) against the u16 millimetres of the same frames: f64(mm)/1000 is
    exactly the u16 path's conversion, so dense and hash states are bit-identical."""
    import torch
    from tsdf_amd import _ffi, grid_fusion, hash_fusion
    d, c, poses = _synth(13, start=520)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    d64 = torch.from_numpy(d.astype(np.float64) / 1000.0).cuda()
    d16 = torch.from_numpy(np.ascontiguousarray(d).view(np.int16)).cuda()
    cc = torch.from_numpy(c).cuda()
    torch.cuda.synchronize()
    outs = []
    for dd, kind in ((d64, _ffi.DEPTH_F64_M), (d16, _ffi.DEPTH_U16_MM)):
        g = grid_fusion.TSDFVolume(np.array(BNDS), 0.04)
        g.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True,
                          depth_kind=kind)
        h = hash_fusion.HashTable(np.array(BNDS), 0.04, 1 << 14)
        h.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True,
                          depth_kind=kind)
        outs.append((g.get_state(), h.get_state()))
    (g64, h64), (g16, h16) = outs
    for a, b, x in zip(g64, g16, h64):
        assert _same(a, b) and _same(x, b)
    for a, b in zip(h16, g16):
        assert _same(a, b)


def test_pool_growth_falls_back_whole_when_one_mapping_fails(monkeypatch):
    """The pool's five arrays grow together or not at all: a mapping refused for the fourth
    array (TSDF_HASH_VMM_FAIL=3, a test hook) unmaps the three grown before it, and the pool moves
    to plain allocations by copy -- the result still equals the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion
    monkeypatch.setenv("TSDF_HASH_VMM_FAIL", "3")
    d, c, poses = _synth(24, start=100)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.04, 1 << 12, max_blocks=256)
    h.integrate_batch(d, c, K, Tinv)
    assert h.info()["pool_capacity"] > 256 and h.stats()["bricks_skipped"] > 0
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.04)
    g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


def test_trim_hands_pool_memory_back_and_growth_resumes(monkeypatch):
    """After an asynchronous run (whose pool growth stays ahead of the launches in flight),
    HashTable.trim() compacts the pool into fresh mapped ranges of its allocated blocks plus ~3 %
    (whole 8 MB pieces);
    integration afterwards grows it again, and the state equals the dense grid throughout."""
    from tsdf_amd import grid_fusion, hash_fusion
    d, c, poses = _synth(64, start=100)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 16, max_blocks=1 << 12)  # 512^3: 2^18 bricks
    h.integrate_batch(d[:8], c[:8], K, Tinv[:8])  # synchronous start (reports lag two launches)
    h.integrate_batch(d[8:40], c[8:40], K, Tinv[8:40], sync=False)
    h.sync()
    before = h.info()
    assert before["pool_mapped"] == 1, before
    h.trim()
    after = h.info()
    per_piece = (8 << 20) // (4 * 512)  # blocks in one 8 MB piece of a state array
    top = after["blocks_in_pool"]
    assert after["pool_capacity"] <= before["pool_capacity"]
    assert top <= after["pool_capacity"] <= top + max(256, top // 32) + per_piece
    h.integrate_batch(d[40:], c[40:], K, Tinv[40:])
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)
    assert h.stats()["bricks_skipped"] == 0 or h.info()["pool_capacity"] > after["pool_capacity"]


def test_async_hash_growth_survives_a_turn_into_unseen_space():
    """Advisor r03: asynchronous pool growth must not lag a growth spike.  A camera on the scene's
    sphere-free ring looks along the ring one way (eight frames, integrated once synchronously
    and then five more times asynchronously: no new blocks, so the recent growth is zero), then
    turns to look the other way (as far, as wide, all of it unseen: the whole list is new blocks).
    The room kept for the launches in flight covers two of the cull's brick lists besides the
    recent growth, so nothing is skipped (a skip raises TSDF_E_CAPACITY at the sync) and the
    result equals the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion, scene
    c, R = 5.12, 0.34 * 10.24
    eye = np.array([c + R, c, c])
    poses = []
    for k in range(16):  # 8 looking +y, then 8 looking -y (small target jitter within each)
        sgn = 1.0 if k < 8 else -1.0
        poses.append(scene.look_at(eye, eye + np.array([0.02 * (k % 4), sgn * 5.0, 0.01 * (k % 3)])))
    poses = np.stack(poses)
    dd, cc = scene.render(poses, scene.make_spheres(0), seed=0, start=900)
    dd, cc = np.ascontiguousarray(dd.numpy()), np.ascontiguousarray(cc.numpy())
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    idx = list(range(8)) * 6 + list(range(8, 16)) * 2  # steady x 6 (first one synchronous), turn x 2
    d, col, Tinv = dd[idx], cc[idx], np.linalg.inv(poses[idx])
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 16, max_blocks=1 << 12)
    h.integrate_batch(d[:8], col[:8], K, Tinv[:8])  # synchronous start (its overflows re-run exactly)
    skipped0 = h.stats()["bricks_skipped"]
    used0 = h.info()["used"]
    h.integrate_batch(d[8:48], col[8:48], K, Tinv[8:48], sync=False)
    h.sync()
    used1 = h.info()["used"]
    h.integrate_batch(d[48:], col[48:], K, Tinv[48:], sync=False)
    h.sync()  # raises TSDF_E_CAPACITY if a launch in flight ran out of pool
    assert h.stats()["bricks_skipped"] == skipped0
    assert used1 == used0 and h.info()["used"] - used1 > used0 / 2  # steady, then a spike
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    g.integrate_batch(d, col, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


def test_trim_integrate_trim_integrate_stays_exact():
    """Advisor r03: every trim compacts the pool into fresh address ranges and retires the old ones
    (kept reserved until the handle is destroyed, never handed out again); trim / integrate cycles
    keep the state bit-identical to the dense grid."""
    from tsdf_amd import grid_fusion, hash_fusion
    d, c, poses = _synth(48, start=200)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 16, max_blocks=1 << 12)
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    h.integrate_batch(d[:8], c[:8], K, Tinv[:8])
    for k in range(1, 6):
        lo, hi = 8 * k, 8 * (k + 1)
        h.integrate_batch(d[lo:hi], c[lo:hi], K, Tinv[lo:hi], sync=(k % 2 == 0))
        h.trim()
        h.trim()  # a second trim in a row: nothing to gain, nothing changes
    g.integrate_batch(d, c, K, Tinv)
    assert h.info()["pool_mapped"] == 1
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)


def test_long_per_frame_hash_run_doubles_only_with_its_keys():
    """Round-5 verdict item 4: 2048 per-frame deferred calls (256 bench-ring frames, f64 metres,
    cycled 8 times) into a table of 2^10 at 4 cm.  Every 8-frame batch ends by freeing the blocks
    its cull inserted for bricks no frame updated -- tombstones where the next slot is taken -- so
    over the run the table sees thousands of them.  The table must double only as its live keys
    require (needs_resize / double_table_size, hash_fusion.py:156-161,414-437): the last doubling
    was due when the live keys reached 0.75 of the size before it; tombstones are purged by
    same-size rebuilds and stay within the policy's limit.  The state equals the dense grid."""
    import torch
    from tsdf_amd import grid_fusion, hash_fusion, scene
    n, cycles = 256, 8
    poses = scene.trajectory(n, seed=0, radius_frac=scene.BENCH_RING)
    dd, cc = scene.render(poses, scene.make_spheres(0, ring_frac=scene.BENCH_RING), seed=0,
                          device=torch.device("cuda", 0), depth_dtype=torch.int16)
    d = np.ascontiguousarray(dd.cpu().numpy().view(np.uint16))
    c = np.ascontiguousarray(cc.cpu().numpy())
    del dd, cc
    K = scene.intrinsics()
    m = d.astype(np.float64) / 1000.0  # as grid_demo1.py:81 (millimetre-exact: staged as u16)
    s0 = 1 << 10
    h = hash_fusion.HashTable(np.array(BNDS), 0.04, s0, max_blocks=1 << 10)
    caps = [s0]
    grew_in_cycle = []
    for k in range(cycles):
        for f in range(n):
            h.integrate(c[f], m[f], K, poses[f])
            if f % 64 == 63:
                i = h.info()
                if i["capacity"] != caps[-1]:
                    caps.append(int(i["capacity"]))
                    grew_in_cycle.append(k)
    h.sync()
    info = h.info()
    ms, live = int(info["capacity"]), int(info["used"])
    # the policy's size for the run's keys: the start size doubled while live >= 0.75 of it (the
    # keys at a check include the batch's not-yet-freed inserts: up to a few hundred more)
    need = s0
    while live >= 0.75 * need:
        need *= 2
    assert ms in (need, 2 * need), (ms, need, live, caps)
    if ms == 2 * need:  # only if the transient inserts crossed the threshold at a check
        assert live + 2048 >= 0.75 * need, (ms, need, live)
    # the table grows only during the first pass over the frames (afterwards no new keys; the
    # tombstones each call leaves are purged at the table's size), by whole doublings
    assert grew_in_cycle and max(grew_in_cycle) == 0, (caps, grew_in_cycle)
    assert all(b > a and (b // a) & (b // a - 1) == 0 for a, b in zip(caps, caps[1:])), caps
    assert info["tombstones"] + live < 0.75 * ms + 2048, info  # purged, within one call's frees
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.04)
    Tinv = np.linalg.inv(poses)
    for k in range(cycles):
        g.integrate_batch(d, c, K, Tinv)
    for a, b in zip(g.get_state(), h.get_state()):
        assert np.array_equal(a, b)
