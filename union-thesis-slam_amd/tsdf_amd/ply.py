"""PLY writers of the reference (grid_fusion.py:386-446, meshwrite / pcwrite): ASCII PLY with the
same header and per-line formats ("%f" coordinates and normals, "%d" colours, "3 i j k"
faces), so files written from this build's meshes open wherever the reference's do."""
from __future__ import annotations

import numpy as np


def _header(n_verts, props, n_faces=None):
    lines = ["ply", "format ascii 1.0", f"element vertex {n_verts}"]
    lines += [f"property {t} {n}" for t, n in props]
    if n_faces is not None:
        lines += [f"element face {n_faces}", "property list uchar int vertex_index"]
    lines.append("end_header")
    return "\n".join(lines) + "\n"


def meshwrite(filename, verts, faces, norms, colors):
    """grid_fusion.py:386-418."""
    verts, faces, norms = np.asarray(verts), np.asarray(faces), np.asarray(norms)
    colors = np.asarray(colors)
    props = [("float", a) for a in ("x", "y", "z", "nx", "ny", "nz")] + [("uchar", a) for a in ("red", "green", "blue")]
    with open(filename, "w") as fh:
        fh.write(_header(verts.shape[0], props, faces.shape[0]))
        for v, n, c in zip(verts, norms, colors):
            fh.write("%f %f %f %f %f %f %d %d %d\n" % (v[0], v[1], v[2], n[0], n[1], n[2], c[0], c[1], c[2]))
        for f in faces:
            fh.write("3 %d %d %d\n" % (f[0], f[1], f[2]))


def pcwrite(filename, xyzrgb):
    """grid_fusion.py:421-446."""
    xyzrgb = np.asarray(xyzrgb)
    xyz, rgb = xyzrgb[:, :3], xyzrgb[:, 3:].astype(np.uint8)
    props = [("float", a) for a in ("x", "y", "z")] + [("uchar", a) for a in ("red", "green", "blue")]
    with open(filename, "w") as fh:
        fh.write(_header(xyz.shape[0], props))
        for p, c in zip(xyz, rgb):
            fh.write("%f %f %f %d %d %d\n" % (p[0], p[1], p[2], c[0], c[1], c[2]))
