"""GPU marching cubes (tsdf_dense_extract_mesh) against the oracle's
restatement (oracle/mc_oracle.py): vertices, colours and faces bit-exact, normals within 1e-6.
Triangulation parity with the reference's skimage.marching_cubes_lewiner is UNPINNED (skimage is
not installed); the vertex rule (linear zero crossings on grid edges, colours of the voxels at
round(vertex), grid_fusion.py:336-346) is the reference's."""
import numpy as np
import pytest

from conftest import load_lounge, lounge_intrinsics
import mc_oracle

pytestmark = pytest.mark.gpu
C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]


@pytest.fixture(scope="module")
def gf():
    from tsdf_amd import grid_fusion
    return grid_fusion


def _check(vol, t, c):
    v, n, col, f = vol.extract_mesh()
    rv, rn, rc, rf = mc_oracle.extract(t, c, vol._vol_origin, vol._voxel_size)
    assert v.shape == rv.shape and f.shape == rf.shape
    assert np.array_equal(v.view(np.uint32), rv.view(np.uint32))
    assert np.array_equal(col, rc) and np.array_equal(f, rf)
    assert np.abs(n - rn).max() <= 1e-6
    return v, n, col, f


def test_mesh_of_lounge_c1_equals_oracle(gf):
    K = lounge_intrinsics()
    vol = gf.TSDFVolume(np.array(C1), 0.04)
    for i in range(3):
        _, depth, rgb, pose = load_lounge(i)
        vol.integrate(rgb, depth, K, pose)
    t, _, c = vol.get_state()
    v, n, col, f = _check(vol, t, c)
    assert len(f) > 10000
    verts, faces, norms, colors = vol.get_mesh()  # the reference's return order
    assert np.array_equal(verts, v) and np.array_equal(faces, f) and np.array_equal(colors, col)
    pc = vol.get_point_cloud()
    assert pc.shape == (len(v), 6) and np.array_equal(pc[:, :3], v) and np.array_equal(pc[:, 3:], col)


def test_mesh_of_ragged_set_state_volume(gf):
    """A state written with set_state into a volume whose dims are not multiples of 8, with
    exact zeros and both signs at the borders."""
    rng = np.random.default_rng(5)
    bnds = np.array([[0.0, 0.63], [0.0, 0.45], [0.0, 0.37]])
    vol = gf.TSDFVolume(bnds.copy(), 0.01)
    shape = tuple(int(d) for d in vol._vol_dim)
    x, y, z = np.meshgrid(*(np.arange(s) for s in shape), indexing="ij")
    t = np.clip((np.sqrt((x - 30.3) ** 2 + (y - 20.2) ** 2 + (z - 18.9) ** 2) - 14.0) / 4.0, -1, 1).astype(np.float32)
    t[::7, ::5, ::3] = 0.0
    c = rng.integers(0, 1 << 24, size=shape).astype(np.float32)
    vol.set_state(t, np.ones(shape, np.float32), c)
    _check(vol, t, c)


def test_hash_mesh_equals_dense_mesh(gf):
    from tsdf_amd import hash_fusion
    K = lounge_intrinsics()
    vol = gf.TSDFVolume(np.array(C1), 0.04)
    ht = hash_fusion.HashTable(np.array(C1), 0.04, 1 << 16)
    for i in range(2):
        _, depth, rgb, pose = load_lounge(i)
        vol.integrate(rgb, depth, K, pose)
        ht.integrate(rgb, depth, K, pose)
    a, b = vol.get_mesh(), ht.get_mesh()
    t_h = ht.get_state()[0]
    if np.array_equal(vol.get_state()[0], t_h):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    else:  # f32 hash state may differ from the grid's by rounding; meshes agree in topology
        assert abs(len(a[0]) - len(b[0])) <= 0.001 * len(a[0])


def test_hash_densifies_on_the_device_like_the_host_export(gf):
    """tsdf_hash_to_dense (get_mesh / get_point_cloud of the hash without a host round trip)
    writes exactly get_state()'s volume into a dense handle: integrated blocks, an entry of
    weight 0 set by add_entries, a removed entry, and a ragged extent (dims not multiples of 8)."""
    from tsdf_amd import _ffi, hash_fusion
    bnds = np.array([[-2.56, 1.48], [-2.52, 2.56], [0.0, 5.00]])
    K = lounge_intrinsics()
    ht = hash_fusion.HashTable(bnds.copy(), 0.04, 1 << 12)
    for i in range(2):
        _, depth, rgb, pose = load_lounge(i)
        ht.integrate(rgb, depth, K, pose)
    ht.add_entries([[1, 2, 3], [100, 126, 124]], tsdf=[0.5, -0.25], weight=[0.0, 3.0], color=[7.0, 65793.0])
    ht.remove_entries([[1, 2, 4]])
    grid = ht._as_grid()
    for a, b in zip(grid.get_state(), ht.get_state()):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    other = gf.TSDFVolume(np.array(C1), 0.04)
    with pytest.raises(_ffi.TSDFError):
        _ffi.call("tsdf_hash_to_dense", ht._h, other._h)  # dims differ
