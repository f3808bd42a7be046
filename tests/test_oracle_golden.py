"""Pin the CPU oracle (oracle/) to golden vectors produced by the reference itself.

Fixtures come from tools/gen_golden.py (the reference imported in the build container with
numba-typing-faithful helpers).  Everything here runs on the CPU.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, load_lounge, lounge_intrinsics
import oracle as O
from bucket_table import BucketTable, hash_value


def _state(vol):
    w = vol._weight_vol_cpu.reshape(-1)
    idx = np.flatnonzero(w > 0)
    return idx, vol._tsdf_vol_cpu.reshape(-1)[idx], w[idx], vol._color_vol_cpu.reshape(-1)[idx]


def test_hash_kat_int64_int32():
    g = np.load(os.path.join(GOLD, "hash_kat.npz"))
    for si, n in enumerate(g["sizes"]):
        assert np.array_equal(O.hash_keys(g["coords"], int(n), 64), g["h64"][si])
        assert np.array_equal(O.hash_keys(g["coords"], int(n), 32), g["h32"][si])
    # hash_demo1.py:141-147 printed values and the SURVEY's int32/int64 example
    assert list(O.hash_keys([[333, 234, 241], [342, 234, 241], [332, 234, 242]], 100000)) == [53356, 5995, 83120]
    assert O.hash_keys([[80, 56, 0]], 100000, 64)[0] == 58888
    assert O.hash_keys([[80, 56, 0]], 100000, 32)[0] == 91592
    # the scalar restatement used by the bucket emulator agrees
    for c in g["coords"][:32]:
        assert hash_value(c, 1000000, 32) == O.hash_keys([c], 1000000, 32)[0]
        assert hash_value(c, 1000000, 64) == O.hash_keys([c], 1000000, 64)[0]


@pytest.mark.parametrize("name", ["dense_c1", "dense_c1_ow"])
def test_dense_oracle_matches_reference_bit_exact(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    bnds = np.array([[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]])
    vol = O.OracleTSDFVolume(bnds, 0.04)
    assert np.array_equal(vol._vol_dim, g["dims"]) and np.array_equal(vol._vol_origin, g["origin"])
    assert np.array_equal(bnds, g["bounds_after"])  # the vol_bnds[:,1] rewrite quirk
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        n = vol.integrate(rgb, depth, K, pose, obs_weight=float(g["obs_weight"][f]))
        assert n == int(g["f%d_nupd" % f])
        idx, t, w, c = _state(vol)
        assert np.array_equal(idx, g["f%d_idx" % f])
        assert np.array_equal(t.view(np.uint32), g["f%d_tsdf" % f].view(np.uint32))
        assert np.array_equal(w, g["f%d_weight" % f])
        assert np.array_equal(c, g["f%d_color" % f])


def test_lounge_decode_is_the_fixture_decode():
    """The fixtures were made from PIL-decoded frames; make sure this PIL decodes identically."""
    import hashlib
    with open(os.path.join(GOLD, "lounge", "decoded_sha256.json")) as f:
        shas = json.load(f)
    for i in range(3):
        d, _, rgb, _ = load_lounge(i)
        assert hashlib.sha256(d.tobytes()).hexdigest() == shas["frame-%06d.depth" % i]
        assert hashlib.sha256(rgb.tobytes()).hexdigest() == shas["frame-%06d.color" % i]


def test_hash_oracle_matches_reference_hash_path():
    """HashTable.integrate (per-voxel f64 Voxel loop) vs the oracle's hash restatement."""
    g = np.load(os.path.join(GOLD, "hash_c1.npz"))
    hv = O.OracleHashVolume(np.array([[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]), 0.04)
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        hv.integrate(rgb, depth, K, pose, obs_weight=3.0)  # ignored, like hash_fusion.py:141,145
        idx, sdf, w, c = hv.entries()
        pos = np.stack(np.unravel_index(idx, tuple(hv._vol_dim)), 1)
        assert np.array_equal(pos, g["f%d_pos" % f])
        assert np.array_equal(sdf, g["f%d_sdf" % f])
        assert np.array_equal(w, g["f%d_weight" % f])
        assert np.array_equal(c, g["f%d_color" % f])
        assert len(idx) == int(g["f%d_entries" % f])


def test_hash_and_grid_paths_agree():
    """same voxel set and colour, tsdf within ~1e-7 (f64 vs f32 state)."""
    gd = np.load(os.path.join(GOLD, "dense_c1.npz"))
    gh = np.load(os.path.join(GOLD, "hash_c1.npz"))
    dims = tuple(gd["dims"])
    pos = np.ravel_multi_index(gh["f2_pos"].T, dims)
    assert np.array_equal(pos, gd["f2_idx"])
    assert np.array_equal(gh["f2_color"], gd["f2_color"].astype(np.float64))
    assert np.abs(gh["f2_sdf"] - gd["f2_tsdf"]).max() < 1e-6


def test_synthetic_frames_bit_exact():
    g = np.load(os.path.join(GOLD, "synth_c1.npz"))
    vol = O.OracleTSDFVolume(np.array([[0.0, 10.24]] * 3), 0.08)
    for f in range(2):
        d = g["depth_u16"][f].astype(float) / 1000.0
        n = vol.integrate(g["rgb"][f], d, g["K"], g["poses"][f])
        assert n == int(g["f%d_nupd" % f])
        idx, t, w, c = _state(vol)
        assert np.array_equal(idx, g["f%d_idx" % f])
        assert np.array_equal(t.view(np.uint32), g["f%d_tsdf" % f].view(np.uint32))
        assert np.array_equal(w, g["f%d_weight" % f])
        assert np.array_equal(c, g["f%d_color" % f])


def _lounge2cm_run(n_frames):
    with open(os.path.join(GOLD, "lounge2cm_kat.json")) as fh:
        kat = json.load(fh)
    hv = O.OracleTSDFVolume(np.array(kat["bounds"]), kat["voxel_size"])
    K = lounge_intrinsics()
    new_keys = []
    for f in range(n_frames):
        _, depth, _, pose = load_lounge(f, color=False)
        before = hv._weight_vol_cpu.reshape(-1) > 0
        n = hv.integrate(np.zeros(depth.shape + (3,), np.uint8), depth, K, pose)
        after = hv._weight_vol_cpu.reshape(-1) > 0
        nk = np.flatnonzero(after & ~before)
        assert n == kat["frames"][f]["updated"]
        assert len(nk) == kat["frames"][f]["new_keys"]
        new_keys.append(np.stack(np.unravel_index(nk, tuple(hv._vol_dim)), 1))
    return kat, hv, new_keys


@pytest.mark.slow
def test_lounge_2cm_ten_frames_counts_digest_and_author_kats():
    """G3: per-frame updated/new-key counts, the final-state digest, and the author's own
    recorded numba run (hash_fusion_demos/cProfile): 354,383 updates in frame 0,
    Σweight 3,557,017 and 389,590 unique keys after ten frames."""
    import hashlib
    kat, vol, new_keys = _lounge2cm_run(10)
    assert kat["frames"][0]["updated"] == 354383
    assert sum(f["updated"] for f in kat["frames"]) == 3557017
    assert int(vol._weight_vol_cpu.sum(dtype=np.float64)) == 3557017
    idx = np.flatnonzero(vol._weight_vol_cpu.reshape(-1) > 0)
    assert len(idx) == kat["unique"] == 389590
    h = hashlib.sha256()
    for a in (idx.astype(np.int64), vol._tsdf_vol_cpu.reshape(-1)[idx], vol._weight_vol_cpu.reshape(-1)[idx]):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == kat["digest_idx_tsdf_weight"]

    # Replay the reference's chained-bucket insertion on those keys (n = 10^6): the author's
    # run created 298,500 buckets and 0 overflow chains in frame 0, 322,698 and 4 after ten
    # frames -- only with int32-wrapping keys (int64 gives 298,252/2 and 322,454/3).
    for bits, want0, want10 in ((32, (298500, 0), (322698, 4)), (64, (298252, 2), (322454, 3))):
        bt = BucketTable(1000000, int_bits=bits)
        for f, keys in enumerate(new_keys):
            for k in keys:
                bt.add(k)
            if f == 0:
                assert (bt.buckets_created, bt.overflows) == want0
        assert (bt.buckets_created, bt.overflows) == want10
        assert bt.count_entries() == 389590


@pytest.mark.slow
def test_lounge_512_frame0_digest():
    import hashlib
    with open(os.path.join(GOLD, "lounge512_kat.json")) as fh:
        kat = json.load(fh)
    vol = O.OracleTSDFVolume(np.array(kat["bounds"]), kat["voxel_size"])
    _, depth, rgb, pose = load_lounge(0)
    assert vol.integrate(rgb, depth, lounge_intrinsics(), pose) == kat["updated"] == 354352
    idx = np.flatnonzero(vol._weight_vol_cpu.reshape(-1) > 0)
    h = hashlib.sha256()
    for a in (idx.astype(np.int64), vol._tsdf_vol_cpu.reshape(-1)[idx],
              vol._weight_vol_cpu.reshape(-1)[idx], vol._color_vol_cpu.reshape(-1)[idx]):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == kat["digest_idx_tsdf_weight_color"]


def test_oracle_view_frustum_matches_reference_over_1000_frames():
    """G6: the oracle's get_view_frustum (grid_fusion.py:371-383, dgemm FMA chain) equals the
    reference's output bit for bit on all 1000 lounge frames, and the demo's running min/max
    (grid_demo1.py:50-64) reproduces the bounds the reference's tests hard-code
    (tests/hash_map_test.py:11, printed to 8 digits)."""
    g = np.load(os.path.join(GOLD, "frustum_bounds.npz"))
    H, W = (int(x) for x in g["shape"])
    md = g["max_depth_mm"] / 1000.0
    for i in range(0, 1000, 7):
        v = O.view_frustum(md[i], H, W, g["intr"], g["poses"][i])
        assert np.array_equal(v.view(np.uint64), g["frustum_pts"][i].view(np.uint64)), i
    b = O.frustum_bounds(md, H, W, g["intr"], g["poses"])
    assert np.array_equal(b, g["bounds"])
    kat = np.array([[-4.22106438, 3.86798203], [-2.6663104, 2.60146141], [0., 5.76272371]])
    assert np.abs(b - kat).max() < 1e-8


@pytest.mark.parametrize("name", ["dense_c1", "dense_c1_ow"])
def test_numpy_port_matches_reference_fixture(name):
    """bench.py's NumPy CPU baseline (oracle.numpy_port_integrate, the reference's own
    full-volume structure) reproduces the reference fixture bit for bit."""
    g = np.load(os.path.join(GOLD, name + ".npz"))
    vol = O.OracleTSDFVolume(np.array([[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]), 0.04)
    coords = O.vox_coords_for(vol._vol_dim)
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        n = O.numpy_port_integrate(vol, coords, rgb, depth, K, pose, obs_weight=float(g["obs_weight"][f]))
        assert n == int(g["f%d_nupd" % f])
        idx, t, w, c = _state(vol)
        assert np.array_equal(idx, g["f%d_idx" % f])
        assert np.array_equal(t.view(np.uint32), g["f%d_tsdf" % f].view(np.uint32))
        assert np.array_equal(w, g["f%d_weight" % f]) and np.array_equal(c, g["f%d_color" % f])


@pytest.mark.slow
def test_numpy_port_hash_matches_reference_hash_path():
    """bench.py's hash CPU baseline (oracle.NumpyPortHash: the per-voxel loop of
    hash_fusion.py:134-145 over the chained-bucket table, float64 Voxel state) reproduces the
    reference's hash fixture exactly, table statistics included."""
    g = np.load(os.path.join(GOLD, "hash_c1.npz"))
    hp = O.NumpyPortHash(np.array([[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]), 0.04, 1000000)
    coords = O.vox_coords_for(hp._vol_dim)
    K = lounge_intrinsics()
    for f in range(3):
        _, depth, rgb, pose = load_lounge(f)
        hp.integrate(coords, rgb, depth, K, pose)
        t = hp.table
        pos = np.array(t.pos, np.int64)
        order = np.lexsort((pos[:, 2], pos[:, 1], pos[:, 0]))
        assert np.array_equal(pos[order], g["f%d_pos" % f])
        assert np.array_equal(np.array(hp.sdf)[order], g["f%d_sdf" % f])
        assert np.array_equal(np.array(hp.weight)[order], g["f%d_weight" % f])
        assert np.array_equal(np.array(hp.color)[order], g["f%d_color" % f])
        assert t.count_entries() == int(g["f%d_entries" % f])
        assert t.nonempty == int(g["f%d_nonempty" % f]) and t.collisions() == int(g["f%d_collisions" % f])
