"""Dense grid on the GPU vs the reference (golden fixtures) and the oracle -- bit-exact.

Every test here calls the HIP path through the C-ABI (tsdf_amd -> libtsdf_hip.so).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, load_lounge, lounge_intrinsics
import oracle as O

pytestmark = pytest.mark.gpu

C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]


@pytest.fixture(scope="module")
def gf():
    from tsdf_amd import grid_fusion
    return grid_fusion


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def _sparse(vol):
    t, w, c = vol.get_state()
    w = w.reshape(-1)
    idx = np.flatnonzero(w > 0)
    return idx, t.reshape(-1)[idx], w[idx], c.reshape(-1)[idx], (t, w, c)


@pytest.mark.parametrize("name", ["dense_c1", "dense_c1_ow"])
def test_lounge_c1_matches_reference_fixture(gf, name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    bnds = np.array(C1)
    vol = gf.TSDFVolume(bnds, 0.04)
    assert np.array_equal(bnds, g["bounds_after"])  # vol_bnds[:,1] rewritten like the reference
    assert np.array_equal(vol._vol_dim, g["dims"]) and np.array_equal(vol._vol_origin, g["origin"])
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        vol.integrate(rgb, depth, K, pose, obs_weight=float(g["obs_weight"][f]))
        idx, t, w, c, (T, W, C) = _sparse(vol)
        assert np.array_equal(idx, g["f%d_idx" % f])
        assert _same(t, g["f%d_tsdf" % f])
        assert _same(w, g["f%d_weight" % f])
        assert _same(c, g["f%d_color" % f])
        # untouched voxels keep the initial state (grid_fusion.py:52-55)
        assert np.count_nonzero(T.reshape(-1) != 1.0) == np.count_nonzero(g["f%d_tsdf" % f] != 1.0)
    assert vol.stats()["voxel_updates"] == sum(int(g["f%d_nupd" % f]) for f in range(3))
    tv, cv = vol.get_volume()
    assert tv.shape == tuple(g["dims"]) and cv.dtype == np.float32


def test_synthetic_fixture_and_depth_kinds(gf):
    """u16-exact depth (sent as millimetres) and the same frames as float64 metres that are NOT
    millimetre-exact (sent as f64) must both match the oracle bit for bit."""
    g = np.load(os.path.join(GOLD, "synth_c1.npz"))
    vol = gf.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.08)
    for f in range(2):
        d = g["depth_u16"][f].astype(float) / 1000.0
        vol.integrate(g["rgb"][f], d, g["K"], g["poses"][f])
        idx, t, w, c, _ = _sparse(vol)
        assert np.array_equal(idx, g["f%d_idx" % f])
        assert _same(t, g["f%d_tsdf" % f]) and _same(w, g["f%d_weight" % f]) and _same(c, g["f%d_color" % f])

    # f64 path + float colour path, against the oracle
    rng = np.random.default_rng(5)
    vol2 = gf.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.08)
    orc = O.OracleTSDFVolume(np.array([[0.0, 10.24]] * 3), 0.08)
    for f in range(2):
        d = g["depth_u16"][f].astype(float) / 1000.0 + rng.uniform(0, 1e-4, size=g["depth_u16"][f].shape)
        d[g["depth_u16"][f] == 0] = 0
        col = g["rgb"][f].astype(np.float64) + rng.uniform(0, 0.9, size=g["rgb"][f].shape)  # folded on host
        vol2.integrate(col, d, g["K"], g["poses"][f], obs_weight=0.6)
        orc.integrate(col, d, g["K"], g["poses"][f], obs_weight=0.6)
    T, W, C = vol2.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)


@pytest.mark.parametrize("bounds,vs", [
    ([[-1.3, 1.1], [-0.9, 1.7], [0.3, 4.0]], 0.05),      # dims not multiples of 8
    ([[-0.01, 0.01], [-0.01, 0.01], [2.0, 2.02]], 0.02),  # a single voxel
    ([[-6.0, -5.0], [-6.0, -5.0], [-3.0, -2.0]], 0.05),   # entirely outside the frustum
])
def test_ragged_and_degenerate_volumes(gf, bounds, vs):
    K = lounge_intrinsics()
    vol = gf.TSDFVolume(np.array(bounds, float), vs)
    orc = O.OracleTSDFVolume(np.array(bounds, float), vs)
    for f in range(2):
        _, depth, rgb, pose = load_lounge(f)
        vol.integrate(rgb, depth, K, pose)
        orc.integrate(rgb, depth, K, pose)
    T, W, C = vol.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)


@pytest.mark.parametrize("cxy", [(1280.0, 960.0), (3000.5, -200.25)])
def test_large_image_and_off_centre_principal_point(gf, cxy):
    # 2560x1920 frames (the lounge frame upsampled 4x) with the principal point at the centre or
    # outside the image: the fast pixel path's boundary margin scales with max(W, H) + |c|
    # (frame_margin, csrc/tsdf_device.h), so the classification stays bit-exact
    K = lounge_intrinsics().copy()
    K[0, 0] *= 4.0
    K[1, 1] *= 4.0
    K[0, 2], K[1, 2] = cxy
    vol = gf.TSDFVolume(np.array(C1), 0.04)
    orc = O.OracleTSDFVolume(np.array(C1), 0.04)
    for f in range(2):
        _, depth, rgb, pose = load_lounge(f)
        depth = np.ascontiguousarray(np.repeat(np.repeat(depth, 4, 0), 4, 1))
        rgb = np.ascontiguousarray(np.repeat(np.repeat(rgb, 4, 0), 4, 1))
        vol.integrate(rgb, depth, K, pose)
        orc.integrate(rgb, depth, K, pose)
    T, W, C = vol.get_state()
    assert int((W > 0).sum()) > 0
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)


def test_empty_and_invalid_depth_is_a_no_op(gf):
    K = lounge_intrinsics()
    vol = gf.TSDFVolume(np.array(C1), 0.04)
    _, depth, rgb, pose = load_lounge(0)
    vol.integrate(rgb, np.zeros_like(depth), K, pose)
    # camera looking away from the volume
    away = pose.copy()
    away[:3, 2] *= -1
    away[:3, 0] *= -1
    vol.integrate(rgb, depth, K, away)
    T, W, C = vol.get_state()
    assert vol.stats()["list_errors"] == 0
    orc = O.OracleTSDFVolume(np.array(C1), 0.04)
    orc.integrate(rgb, depth, K, away)
    assert int(W.sum()) == int(orc._weight_vol_cpu.sum())
    assert _same(T, orc._tsdf_vol_cpu)


def test_lounge_512_frame0_digest(gf):
    """G5 at full BASELINE size (512^3 @ 2 cm): count and digest of the reference's result."""
    with open(os.path.join(GOLD, "lounge512_kat.json")) as fh:
        kat = json.load(fh)
    vol = gf.TSDFVolume(np.array(kat["bounds"]), kat["voxel_size"])
    _, depth, rgb, pose = load_lounge(0)
    vol.integrate(rgb, depth, lounge_intrinsics(), pose)
    idx, t, w, c, _ = _sparse(vol)
    assert len(idx) == kat["updated"] == 354352
    h = hashlib.sha256()
    for a in (idx.astype(np.int64), t, w, c):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == kat["digest_idx_tsdf_weight_color"]


def test_lounge_2cm_ten_frames_digest(gf):
    with open(os.path.join(GOLD, "lounge2cm_kat.json")) as fh:
        kat = json.load(fh)
    vol = gf.TSDFVolume(np.array(kat["bounds"]), kat["voxel_size"])
    K = lounge_intrinsics()
    for f in range(10):
        _, depth, _, pose = load_lounge(f, color=False)
        vol.integrate(np.zeros(depth.shape + (3,), np.uint8), depth, K, pose)
        assert vol.stats(reset=True)["voxel_updates"] == kat["frames"][f]["updated"]
    idx, t, w, _, _ = _sparse(vol)
    assert len(idx) == kat["unique"] == 389590
    assert int(w.sum(dtype=np.float64)) == 3557017
    h = hashlib.sha256()
    for a in (idx.astype(np.int64), t, w):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == kat["digest_idx_tsdf_weight"]


def _synth(n, start=0, room=10.24):
    from tsdf_amd import scene
    poses = scene.trajectory(n, seed=0, start=start)
    d, c = scene.render(poses, scene.make_spheres(0), seed=0, start=start)
    return d.numpy(), c.numpy(), poses


def test_batch_equals_sequential_and_oracle(gf):
    d, c, poses = _synth(4)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    seq = gf.TSDFVolume(bnds.copy(), 0.08)
    bat = gf.TSDFVolume(bnds.copy(), 0.08)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    for f in range(4):
        seq.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f])
        orc.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f])
    Tinv = np.linalg.inv(poses)
    bat.integrate_batch(np.ascontiguousarray(d), np.ascontiguousarray(c), K, Tinv)
    A, B = seq.get_state(), bat.get_state()
    for a, b, o in zip(A, B, (orc._tsdf_vol_cpu, orc._weight_vol_cpu, orc._color_vol_cpu)):
        assert _same(a, b) and _same(a, o)


def test_device_resident_batch(gf):
    """Inputs already in HBM (torch tensors), as the bench runs them."""
    torch = pytest.importorskip("torch")
    d, c, poses = _synth(3, start=500)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    vol = gf.TSDFVolume(bnds.copy(), 0.08)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    dd = torch.from_numpy(np.ascontiguousarray(d).view(np.int16)).cuda()  # raw u16 bits
    cc = torch.from_numpy(c).cuda()
    torch.cuda.synchronize()
    vol.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, np.linalg.inv(poses), hw=d.shape[1:],
                        device_ptrs=True)
    for f in range(3):
        orc.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f])
    T, W, C = vol.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)


def test_slab_shards_reassemble_bit_exact(gf):
    """Slab sharding: x-slabs with a global index offset reproduce the
    unsharded volume exactly, including a slab boundary that is not brick aligned."""
    bnds = np.array(C1)
    K = lounge_intrinsics()
    full = gf.TSDFVolume(bnds.copy(), 0.04)
    parts = [gf.TSDFVolume(bnds.copy(), 0.04, slab=s) for s in ((0, 43), (43, 96), (96, 128))]
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        for v in [full] + parts:
            v.integrate(rgb, depth, K, pose)
    F = full.get_state()
    P = [p.get_state() for p in parts]
    for k in range(3):
        assert _same(F[k], np.concatenate([p[k] for p in P], axis=0))


@pytest.mark.parametrize("world", [3, 8])
def test_cyclic_column_shards_reassemble_bit_exact(gf, world):
    """Cyclic brick-column sharding (tsdf_dense_create_shard, the bench's multi-GPU layout):
    every shard equals the unsharded volume's rows at its global x, including a ragged last
    column (X = 101 is not a multiple of 8), for both single-frame and batched integrate."""
    from tsdf_amd import sharding
    bnds = np.array([[-2.56, 1.48], [-2.56, 2.56], [0.0, 5.12]])  # 101 x 128 x 128 @ 4 cm
    K = lounge_intrinsics()
    full = O.OracleTSDFVolume(bnds.copy(), 0.04)
    X = int(full._vol_dim[0])
    assert X == 101
    parts = [gf.TSDFVolume(bnds.copy(), 0.04, shard=(r, world)) for r in range(world)]
    frames = [load_lounge(f) for f in range(3)]
    for _, depth, rgb, pose in frames:
        full.integrate(rgb, depth, K, pose)
    for p in parts:
        p.integrate(frames[0][2], frames[0][1], K, frames[0][3])
        d = np.stack([fr[1] for fr in frames[1:]])
        c = np.stack([fr[2] for fr in frames[1:]])
        p.integrate_batch(d, c, K, np.linalg.inv(np.stack([fr[3] for fr in frames[1:]])))
    seen = np.zeros(X, int)
    for r, p in enumerate(parts):
        xi = sharding.columns(r, world, X)
        assert np.array_equal(p.x_index, xi)
        seen[xi] += 1
        T, W, C = p.get_state()
        assert _same(T, full._tsdf_vol_cpu[xi]) and _same(W, full._weight_vol_cpu[xi])
        assert _same(C, full._color_vol_cpu[xi])
    assert (seen == 1).all()


def test_long_batch_without_host_sync_matches_oracle(gf):
    """72 frames in one async call (launches of 32 + 32 + 8 frames, no host synchronisation
    between them, as in the bench): cross-kernel visibility of the brick state must hold whatever
    XCD a brick lands on from one launch to the next."""
    d, c, poses = _synth(72, start=40)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    vol = gf.TSDFVolume(bnds.copy(), 0.08)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    vol.integrate_batch(np.ascontiguousarray(d), np.ascontiguousarray(c), K, np.linalg.inv(poses), sync=False)
    n = sum(orc.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f]) for f in range(72))
    vol.sync()
    T, W, C = vol.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)
    assert vol.stats()["voxel_updates"] == n
    assert vol.stats()["list_errors"] == 0


def test_host_ingest_staging_slots_equal_device_path(gf, monkeypatch):
    """Frame ingest: 45 host frames (6 batches of 8 over the four staging
    slots, two of them reused) from pageable numpy arrays and from a pinned torch tensor equal
    the device-resident run bit for bit; the call returns with the host arrays no longer needed."""
    import torch
    monkeypatch.setenv("TSDF_BATCH", "8")  # (6 launches of 8 frames: every staging slot in turn)
    d, c, poses = _synth(45, start=5)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    host = gf.TSDFVolume(bnds.copy(), 0.08)
    pinned = gf.TSDFVolume(bnds.copy(), 0.08)
    dev = gf.TSDFVolume(bnds.copy(), 0.08)
    dh, ch = np.ascontiguousarray(d).copy(), np.ascontiguousarray(c).copy()
    host.integrate_batch(dh, ch, K, Tinv, sync=False)
    dh[:] = 0  # the caller may reuse its buffers as soon as the call returns
    ch[:] = 0
    dp = torch.from_numpy(np.ascontiguousarray(d)).pin_memory()
    cp = torch.from_numpy(np.ascontiguousarray(c)).pin_memory()
    pinned.integrate_batch(dp.data_ptr(), cp.data_ptr(), K, Tinv, hw=d.shape[1:], sync=True)
    dd, cc = torch.from_numpy(np.ascontiguousarray(d)).cuda(), torch.from_numpy(np.ascontiguousarray(c)).cuda()
    torch.cuda.synchronize()
    dev.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True)
    host.sync()
    A, B, C = host.get_state(), pinned.get_state(), dev.get_state()
    for a, b, e in zip(A, B, C):
        assert _same(a, e) and _same(b, e)
    assert host.stats()["voxel_updates"] == dev.stats()["voxel_updates"] > 0


def test_invalid_65535_mask_on_device(gf):
    """Raw u16 frames with 65535 pixels + invalid_65535 equal the demos' host masking
    (depth_im[depth_im == 65.535] = 0, grid_demo1.py:82) fed through the oracle."""
    K = lounge_intrinsics()
    bnds = np.array(C1)
    frames = [load_lounge(i) for i in range(3)]
    raw = np.stack([f[0] for f in frames]).astype(np.uint16)
    raw[:, 100:140, 200:260] = 65535
    raw[1, 300:310, :] = 65535
    rgb = np.stack([f[2] for f in frames])
    poses = np.stack([f[3] for f in frames])
    vol = gf.TSDFVolume(bnds.copy(), 0.04)
    vol.integrate_batch(raw, rgb, K, np.linalg.inv(poses), invalid_65535=True)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.04)
    for i in range(3):
        m = raw[i].astype(float) / 1000.0
        m[m == 65.535] = 0
        orc.integrate(rgb[i], m, K, poses[i])
    T, W, Cc = vol.get_state()
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(Cc, orc._color_vol_cpu)
    # without the mask 65.535 m is a valid (far) depth: a different volume
    vol2 = gf.TSDFVolume(bnds.copy(), 0.04)
    vol2.integrate_batch(raw, rgb, K, np.linalg.inv(poses))
    assert not _same(vol2.get_state()[1], W)


@pytest.mark.parametrize("ingest", ["device", "host"])
def test_prep_cull_pipeline_on_and_off_bit_identical(gf, monkeypatch, ingest):
    """u16 + RGB8 calls run as three-stage pipeline launches (k_fused: integrate batch k, cull
    k+1 and prep k+2 in one launch, three buffer sets, four staging slots; tsdf_dense.hip,
    DESIGN.md §6); TSDF_PIPELINE=0 forces the in-line prep / cull / integrate kernels.  Both
    paths over 29 async frames (4 batches of 8: every set and slot reused) with 65535 masking, from
    device and from host memory, equal each other and the oracle bit for bit."""
    import torch
    monkeypatch.setenv("TSDF_BATCH", "8")
    d, c, poses = _synth(29, start=11)
    d = np.ascontiguousarray(d).astype(np.uint16)
    d[3:9, 50:90, 100:200] = 65535
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    dm = np.where(d == 65535, 0, d)
    n = sum(orc.integrate(c[f], dm[f].astype(float) / 1000.0, K, poses[f]) for f in range(len(d)))
    states = []
    for pipe in ("0", "1"):
        monkeypatch.setenv("TSDF_PIPELINE", pipe)
        vol = gf.TSDFVolume(bnds.copy(), 0.08)
        if ingest == "host":
            vol.integrate_batch(d, np.ascontiguousarray(c), K, Tinv, sync=False, invalid_65535=True)
        else:
            dd, cc = torch.from_numpy(d.view(np.int16)).cuda(), torch.from_numpy(np.ascontiguousarray(c)).cuda()
            torch.cuda.synchronize()
            vol.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True,
                                sync=False, invalid_65535=True)
        vol.sync()
        st = vol.stats()
        assert st["voxel_updates"] == n and st["list_errors"] == 0
        states.append(vol.get_state())
    for a, b, e in zip(states[0], states[1], (orc._tsdf_vol_cpu, orc._weight_vol_cpu, orc._color_vol_cpu)):
        assert _same(a, e) and _same(b, e)


@pytest.mark.parametrize("ingest", ["device", "host"])
def test_rgb8_gathered_in_place_equals_the_rgbx_copy(gf, monkeypatch, ingest):
    """RGB8 frames are gathered in place (3-byte-stride buffer loads, frame_bufs) wherever the byte
    after a frame is readable -- the padded staging slots, or a device array with more of the
    call's frames after it; the call's last device frame goes through the prep's packed RGBX copy.
    TSDF_RGB_DIRECT=0 forces the copy for every frame.  Both, through the fused and the in-line
    kernels, over 19 frames (batches of 8) with colours in every byte, equal the oracle bit for bit."""
    import torch
    monkeypatch.setenv("TSDF_BATCH", "8")
    d, c, poses = _synth(19, start=200)
    rng = np.random.default_rng(3)
    c = np.ascontiguousarray(c)
    c[:, ::7, ::5] = rng.integers(0, 256, c[:, ::7, ::5].shape, dtype=np.uint8)  # (all byte values)
    c[:, -1, -1] = (255, 1, 128)  # the last pixel, whose 4-byte load reaches past the frame
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    n = sum(orc.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f]) for f in range(len(d)))
    for pipe in ("0", "1"):
        for direct in ("0", "1"):
            monkeypatch.setenv("TSDF_PIPELINE", pipe)
            monkeypatch.setenv("TSDF_RGB_DIRECT", direct)
            vol = gf.TSDFVolume(bnds.copy(), 0.08)
            if ingest == "host":
                vol.integrate_batch(np.ascontiguousarray(d), c, K, Tinv, sync=False)
            else:
                dd, cc = torch.from_numpy(np.ascontiguousarray(d).view(np.int16)).cuda(), torch.from_numpy(c).cuda()
                torch.cuda.synchronize()
                vol.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True, sync=False)
            vol.sync()
            assert vol.stats()["voxel_updates"] == n, (pipe, direct)
            T, W, C = vol.get_state()
            assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu), (pipe, direct)
            assert _same(C, orc._color_vol_cpu), (pipe, direct)


def test_bench_workload_at_full_size_matches_oracle_rows(gf):
    """The bench's own path at BASELINE size: 512^3 @ 2 cm, 40 synthetic frames resident in HBM,
    one async call (a full 32-frame batch and an 8-frame one through the three-stage k_fused
    launches).  22 x-rows spread
    over the volume (every residue mod 8, so every lane column of a brick) are checked bit-exact
    against the oracle restricted to those rows; the hash path over the same frames must hold
    the same state on those rows."""
    torch = pytest.importorskip("torch")
    from tsdf_amd import hash_fusion, scene
    n = 40
    d, c, poses = _synth(n, start=120)
    K = scene.intrinsics()
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    dd = torch.from_numpy(np.ascontiguousarray(d).view(np.int16)).cuda()
    cc = torch.from_numpy(np.ascontiguousarray(c)).cuda()
    torch.cuda.synchronize()
    vol = gf.TSDFVolume(bnds.copy(), 0.02)
    assert tuple(int(x) for x in vol._vol_dim) == (512, 512, 512)
    vol.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True, sync=False)
    ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22)
    ht.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True, sync=False)
    vol.sync()
    ht.sync()
    rows = np.arange(5, 512, 23)
    assert len(np.unique(rows % 8)) == 8
    orc = O.OracleTSDFVolume(bnds.copy(), 0.02, x_index=rows)
    n_upd = sum(orc.integrate(c[f], d[f].astype(float) / 1000.0, K, poses[f]) for f in range(n))
    assert n_upd > 1_000_000
    G = [a[rows] for a in vol.get_state()]
    for a, o in zip(G, (orc._tsdf_vol_cpu, orc._weight_vol_cpu, orc._color_vol_cpu)):
        assert _same(a, o)
    Hs = [a[rows] for a in ht.get_state()]
    for a, b in zip(G, Hs):
        assert np.array_equal(a, b)
    sg, sh = vol.stats(), ht.stats()
    assert sg["list_errors"] == 0 and sg["voxel_updates"] == sh["voxel_updates"] > 0


@pytest.mark.parametrize("offset", [(5000.25, -3000.5, 4000.125), (-1.0e4, 2.5e3, -7.5e3)])
def test_volume_far_from_the_world_origin(gf, offset):
    """The bench room moved 5-10 km from the world origin (poses and bounds shifted alike): the
    cull's f32 frustum test is camera-relative and the corner projection starts from f64 lattice
    points, so no voxel the reference updates is culled -- dense and hash equal the oracle (whose
    own f32 world points are coarse out there, 0.5-1 mm) bit for bit."""
    from tsdf_amd import hash_fusion
    d, c, poses = _synth(10, start=210)
    off = np.array(offset)
    poses = poses.copy()
    poses[:, :3, 3] += off
    bnds = np.array([[0.0, 10.24]] * 3) + off[:, None]
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    vol = gf.TSDFVolume(bnds.copy(), 0.08)
    ht = hash_fusion.HashTable(bnds.copy(), 0.08, 1 << 16)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    n = 0
    for f in range(10):
        m = d[f].astype(float) / 1000.0
        vol.integrate(c[f], m, K, poses[f])
        ht.integrate(c[f], m, K, poses[f])
        n += orc.integrate(c[f], m, K, poses[f])
    T, W, C = vol.get_state()
    assert n > 100_000 and vol.stats()["voxel_updates"] == n
    assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu)
    for a, b in zip(ht.get_state(), (T, W, C)):
        assert np.array_equal(a, b)
