"""The texel integrate (DK = 2, round 6): u16 depth + RGB8 gathered as one 8-byte texel per pixel
that the fused launch's prep writes.  The host picks it by the handle's bricks (Base::texel_for);
TSDF_TEXEL=0 / 1 forces it either way, so these tests run both variants on volumes of every size
and require the same bits as the oracle (dense) and as the dense grid (hash).

Every test here calls the HIP path through the C-ABI (tsdf_amd -> libtsdf_hip.so).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def _frames(n, start):
    from tsdf_amd import scene
    poses = scene.trajectory(n, seed=0, start=start)
    d, c = scene.render(poses, scene.make_spheres(0), seed=0, start=start)
    d, c = np.ascontiguousarray(d.numpy()), np.ascontiguousarray(c.numpy())
    rng = np.random.default_rng(11)
    c[:, ::5, ::3] = rng.integers(0, 256, c[:, ::5, ::3].shape, dtype=np.uint8)  # every byte value
    d[:, 40:60, 100:180] = 65535  # invalid under the demos' mask (grid_demo1.py:82)
    return d, c, poses


@pytest.mark.parametrize("ingest", ["device", "host"])
def test_dense_texels_equal_two_gathers_and_oracle(ingest, monkeypatch):
    """21 frames in batches of 8 (full and ragged fused launches) with 65535 masking, through the
    texel kernels and the two-gather kernels: both bit-exact against the oracle."""
    import torch
    from tsdf_amd import grid_fusion
    monkeypatch.setenv("TSDF_BATCH", "8")
    d, c, poses = _frames(21, start=260)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    orc = O.OracleTSDFVolume(bnds.copy(), 0.08)
    n = 0
    for f in range(len(d)):
        m = d[f].astype(float) / 1000.0
        m[m == 65.535] = 0
        n += orc.integrate(c[f], m, K, poses[f])
    assert n > 10_000
    for tex in ("1", "0"):
        monkeypatch.setenv("TSDF_TEXEL", tex)
        vol = grid_fusion.TSDFVolume(bnds.copy(), 0.08)
        if ingest == "host":
            vol.integrate_batch(d, c, K, Tinv, sync=False, invalid_65535=True)
        else:
            dd, cc = torch.from_numpy(d.view(np.int16)).cuda(), torch.from_numpy(c).cuda()
            torch.cuda.synchronize()
            vol.integrate_batch(dd.data_ptr(), cc.data_ptr(), K, Tinv, hw=d.shape[1:], device_ptrs=True,
                                sync=False, invalid_65535=True)
        vol.sync()
        assert vol.stats()["voxel_updates"] == n, tex
        T, W, C = vol.get_state()
        assert _same(T, orc._tsdf_vol_cpu) and _same(W, orc._weight_vol_cpu) and _same(C, orc._color_vol_cpu), tex
        vol.close()


def test_hash_texels_equal_dense_with_exact_reruns(monkeypatch):
    """The hash's fused launches on texels, with a pool small enough that batches overflow and
    re-run exactly (the re-run gathers the batch's texels too), hold the dense grid's state."""
    from tsdf_amd import grid_fusion, hash_fusion
    monkeypatch.setenv("TSDF_BATCH", "8")
    d, c, poses = _frames(17, start=300)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    bnds = np.array([[0.0, 10.24]] * 3)
    Tinv = np.linalg.inv(poses)
    monkeypatch.setenv("TSDF_TEXEL", "0")
    ref = grid_fusion.TSDFVolume(bnds.copy(), 0.08)
    ref.integrate_batch(d, c, K, Tinv, invalid_65535=True)
    G = ref.get_state()
    skipped = []
    for tex in ("1", "0"):
        monkeypatch.setenv("TSDF_TEXEL", tex)
        ht = hash_fusion.HashTable(bnds.copy(), 0.08, 37, max_blocks=16)  # (overflows: exact re-runs)
        ht.integrate_batch(d, c, K, Tinv, invalid_65535=True)
        H = ht.get_state()
        for a, b in zip(G, H):
            assert np.array_equal(a, b), tex
        st = ht.stats()
        assert st["voxel_updates"] == ref.stats()["voxel_updates"] > 0
        skipped.append(st["bricks_skipped"])
        ht.close()
    assert min(skipped) > 0, skipped  # (both variants re-ran skipped bricks)
