"""Mesh extraction on the CPU: the library's case table equals the oracle's restatement of the
rule, the oracle's meshes are closed and consistently oriented, and the PLY writers keep the
reference's format (grid_fusion.py:386-446).  No GPU needed."""
import os

import numpy as np

import mc_oracle
import mc_table


def test_library_case_table_equals_oracle_rule():
    from tsdf_amd import _ffi
    tri = np.zeros(256 * 16, np.int8)
    ntri = np.zeros(256, np.uint8)
    _ffi.call("tsdf_mc_table", _ffi.ptr(tri), _ffi.ptr(ntri))
    ref = np.array(mc_table.table(), np.int8)
    assert np.array_equal(tri.reshape(256, 16), ref)
    assert np.array_equal(ntri, (ref >= 0).sum(axis=1) // 3)
    assert ntri.max() == 5 and ntri[0] == ntri[255] == 0


def _sphere(n=24, r=7.3, c=(11.2, 12.1, 10.7)):
    x, y, z = np.meshgrid(*(np.arange(n),) * 3, indexing="ij")
    d = np.sqrt((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) - r
    return np.clip(d / 3.0, -1, 1).astype(np.float32), np.array(c), r


def test_oracle_mesh_is_closed_and_outward():
    t, c, r = _sphere()
    color = np.full(t.shape, 3 * 65536 + 2 * 256 + 1, np.float32)
    v, n, col, f = mc_oracle.extract(t, color, np.zeros(3, np.float32), 1.0)
    assert len(f) > 100
    # every directed edge once, its reverse once: closed and consistently oriented
    e = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    s = set(map(tuple, e))
    assert len(s) == len(e) and all((b, a) in s for a, b in s)
    assert np.abs(np.linalg.norm(v - c, axis=1) - r).max() < 0.2
    assert (np.einsum("ij,ij->i", n, v - c) > 0).all()
    fn = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    assert (np.einsum("ij,ij->i", fn, v[f].mean(axis=1) - c) > 0).mean() > 0.99
    assert (col == [1, 2, 3]).all()


def test_ply_writers_match_reference_format(tmp_path):
    from tsdf_amd import grid_fusion
    v = np.array([[0.5, 1.25, -2.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]], np.float32)
    n = np.eye(3, dtype=np.float32)
    c = np.array([[255, 0, 7], [1, 2, 3], [9, 8, 7]], np.uint8)
    f = np.array([[0, 1, 2]], np.int32)
    p = os.path.join(tmp_path, "m.ply")
    grid_fusion.meshwrite(p, v, f, n, c)
    lines = open(p).read().splitlines()
    assert lines[:3] == ["ply", "format ascii 1.0", "element vertex 3"]
    assert lines[12:15] == ["element face 1", "property list uchar int vertex_index", "end_header"]
    assert lines[15] == "0.500000 1.250000 -2.000000 1.000000 0.000000 0.000000 255 0 7"
    assert lines[-1] == "3 0 1 2"
    q = os.path.join(tmp_path, "p.ply")
    grid_fusion.pcwrite(q, np.hstack([v, c]))
    lines = open(q).read().splitlines()
    assert lines[2] == "element vertex 3" and lines[9] == "end_header"
    assert lines[10] == "0.500000 1.250000 -2.000000 255 0 7"
