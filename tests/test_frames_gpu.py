"""GPU frame utilities: view-frustum volume bounds through the C-ABI
(tsdf_frustum_bounds) against the oracle and the reference's own fixture (G6)."""
import os

import numpy as np
import pytest

from conftest import GOLD, load_lounge, lounge_intrinsics
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gf():
    from tsdf_amd import grid_fusion
    return grid_fusion


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def test_bounds_1000_lounge_frames_device_resident(gf):
    """All 1000 lounge frames as device-resident u16 images holding each frame's max depth (the
    only pixel get_view_frustum reads), plus a 65535 pixel that the 7-Scenes mask must drop:
    per-frame maxima, every frustum point and the union equal the reference's values bit for
    bit, and the union equals the bounds hard-coded in the reference's tests."""
    import torch
    g = np.load(os.path.join(GOLD, "frustum_bounds.npz"))
    H, W = (int(x) for x in g["shape"])
    n = 1000
    d = torch.zeros((n, H, W), dtype=torch.int16, device="cuda")
    mm = torch.from_numpy(g["max_depth_mm"].astype(np.int64))
    rows = torch.arange(n) % H
    d[torch.arange(n), rows, (torch.arange(n) * 7) % W] = mm.to(torch.int16).cuda()  # u16 bits
    d[:, H - 1, W - 1] = -1  # 65535 mm: invalid under the demos' convention
    torch.cuda.synchronize()
    b, md, pts = gf.view_frustum_bounds(d.data_ptr(), g["intr"], g["poses"], invalid_65535=True,
                                        device_ptrs=True, hw=(H, W), depth_kind=0, n_frames=n,
                                        return_max_depth=True, return_points=True)
    assert np.array_equal(_bits(md), _bits(g["max_depth_mm"] / 1000.0))
    assert np.array_equal(_bits(pts), _bits(g["frustum_pts"]))
    assert np.array_equal(b, g["bounds"])
    assert np.array_equal(_bits(b), _bits(g["bounds_running"][-1]))


def test_bounds_real_lounge_frames_host_u16_and_f64(gf):
    """10 real lounge depth images from host memory, as raw u16 PNG values (7-Scenes mask on
    the device) and as the demos' f64 metres: same maxima, points and bounds as the oracle."""
    K = lounge_intrinsics()
    frames = [load_lounge(i, color=False) for i in range(10)]
    raw = np.stack([f[0] for f in frames]).astype(np.uint16)
    metres = np.stack([f[1] for f in frames])
    poses = np.stack([f[3] for f in frames])
    H, W = raw.shape[1:]
    ref_md = metres.reshape(10, -1).max(axis=1)
    ref_b = O.frustum_bounds(ref_md, H, W, K, poses)
    ref_pts = np.stack([O.view_frustum(ref_md[i], H, W, K, poses[i]) for i in range(10)])
    for depth, inval in ((raw, True), (metres, False)):
        b, md, pts = gf.view_frustum_bounds(depth, K, poses, invalid_65535=inval,
                                            return_max_depth=True, return_points=True)
        assert np.array_equal(_bits(md), _bits(ref_md))
        assert np.array_equal(_bits(pts), _bits(ref_pts))
        assert np.array_equal(b, ref_b)
    # without the mask a 65535 pixel (present in the raw lounge frames) is a 65.535 m depth
    if (raw == 65535).any():
        _, md = gf.view_frustum_bounds(raw, K, poses, return_max_depth=True)
        assert md.max() == 65.535


def test_bounds_init_and_errors(gf):
    from tsdf_amd._ffi import TSDFError
    K = lounge_intrinsics()
    d = np.zeros((1, 48, 64), np.uint16)
    d[0, 3, 5] = 1234
    pose = np.eye(4)
    init = np.array([[-100.0, -99.0], [50.0, 51.0], [0.0, 0.0]])
    b = gf.view_frustum_bounds(d, K, pose[None], init=init)
    ref = O.frustum_bounds([1.234], 48, 64, K, pose[None], init=init)
    assert np.array_equal(b, ref) and b[0, 0] == -100.0 and b[1, 1] == 51.0
    with pytest.raises(ValueError):
        gf.view_frustum_bounds(d.astype(np.float32), K, pose[None])
    with pytest.raises(TSDFError):
        gf.view_frustum_bounds(d, K, pose[None], device=99)
