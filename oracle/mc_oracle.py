"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of the build's marching-cubes extraction, the
checker for tsdf_dense_extract_mesh (csrc/tsdf_mesh.hip).

What the reference does (grid_fusion.py:322-360): skimage.measure.marching_cubes_lewiner(tsdf,
level=0), verts * voxel_size + origin, colours of the voxels at round(verts) decoded to uint8.
skimage is absent here, so the triangulation is PARITY UNPINNED against the reference; what
this file pins is the build's own definition, stated so a reader can check it line by line:

  * a grid edge carries a vertex when exactly one of its end values is < 0;
  * vertex = lower end + t along the edge, t = (0 - v1) / (v2 - v1) in float32;
  * world = vertex * f32(voxel_size) + origin, float32 multiply then add (NumPy 2 keeps a
    float32 array times a Python float in float32);
  * colour = the voxel at np.round(vertex), decoded as grid_fusion.py:341-346 in float32;
  * normal = normalised linear interpolation of central-difference gradients (indices clamped),
    pointing towards positive tsdf;
  * vertices in C-order of (voxel, axis); faces from mc_table, written (0, 2, 1).
"""
from __future__ import annotations

import numpy as np

import mc_table

_F = np.float32


def _grad(t):
    g = np.zeros(t.shape + (3,), _F)
    for a in range(3):
        hi = np.take(t, np.minimum(np.arange(t.shape[a]) + 1, t.shape[a] - 1), axis=a)
        lo = np.take(t, np.maximum(np.arange(t.shape[a]) - 1, 0), axis=a)
        g[..., a] = hi - lo
    return g


def extract(tsdf, color, origin, voxel_size):
    """(verts (N,3) f32 world, normals (N,3) f32, colors (N,3) u8, faces (M,3) i32)."""
    t = np.ascontiguousarray(tsdf, _F)
    X, Y, Z = t.shape
    inside = t < 0
    flags = np.zeros((X, Y, Z, 3), bool)
    flags[:-1, :, :, 0] = inside[:-1] != inside[1:]
    flags[:, :-1, :, 1] = inside[:, :-1] != inside[:, 1:]
    flags[:, :, :-1, 2] = inside[:, :, :-1] != inside[:, :, 1:]
    flat = np.flatnonzero(flags.reshape(-1))
    vox, axis = np.divmod(flat, 3)
    x, y, z = np.unravel_index(vox, (X, Y, Z))
    step = np.eye(3, dtype=np.int64)[axis]
    x2, y2, z2 = x + step[:, 0], y + step[:, 1], z + step[:, 2]
    v1, v2 = t[x, y, z], t[x2, y2, z2]
    tt = (_F(0) - v1) / (v2 - v1)
    p = np.stack([x, y, z], 1).astype(_F)
    p[np.arange(len(p)), axis] = p[np.arange(len(p)), axis] + tt
    verts = p * _F(voxel_size) + np.asarray(origin, _F)
    g = _grad(t)
    g1, g2 = g[x, y, z], g[x2, y2, z2]
    n = g1 + tt[:, None] * (g2 - g1)
    ln = np.sqrt(n[:, 0] * n[:, 0] + n[:, 1] * n[:, 1] + n[:, 2] * n[:, 2])
    with np.errstate(invalid="ignore", divide="ignore"):
        normals = np.where(ln[:, None] > 0, n / ln[:, None], _F(0)).astype(_F)
    r = np.round(p).astype(np.int64)
    cv = np.asarray(color, _F)[r[:, 0], r[:, 1], r[:, 2]]
    cb = np.floor(cv / _F(65536))
    cg = np.floor((cv - cb * _F(65536)) / _F(256))
    cr = cv - cb * _F(65536) - cg * _F(256)
    colors = np.floor(np.stack([cr, cg, cb], 1)).astype(np.uint8)

    # vertex id of grid edge (voxel, axis)
    vid = np.full(X * Y * Z * 3, -1, np.int64)
    vid[flat] = np.arange(len(flat))
    tab = mc_table.table()
    cube = np.zeros((X - 1, Y - 1, Z - 1), np.int64) if min(X, Y, Z) > 1 else np.zeros((0, 0, 0), np.int64)
    for c in range(8):
        ox, oy, oz = c & 1, (c >> 1) & 1, (c >> 2) & 1
        cube |= inside[ox:X - 1 + ox, oy:Y - 1 + oy, oz:Z - 1 + oz].astype(np.int64) << c
    cells = np.argwhere((cube > 0) & (cube < 255))  # C-order
    faces = []
    for cx, cy, cz in cells:
        row = tab[cube[cx, cy, cz]]
        for k in range(0, 15, 3):
            if row[k] < 0:
                break
            ids = []
            for e in row[k:k + 3]:
                a, b = mc_table.EDGES[e]
                ax = (a ^ b).bit_length() - 1
                gx, gy, gz = cx + (a & 1), cy + ((a >> 1) & 1), cz + ((a >> 2) & 1)
                ids.append(vid[((gx * Y + gy) * Z + gz) * 3 + ax])
            faces.append((ids[0], ids[2], ids[1]))
    faces = np.array(faces, np.int32).reshape(-1, 3)
    return verts.astype(_F), normals, colors, faces
