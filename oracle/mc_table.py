"""TEST INFRASTRUCTURE ONLY -- the marching-cubes case table restated for the oracle.

The reference meshes with skimage.measure.marching_cubes_lewiner (grid_fusion.py:327,348), which
is not installed here, so its triangles cannot be reproduced; PARITY UNPINNED for triangles (see
DESIGN.md).  The MI355X build derives its case table from one rule, restated here independently
of the library's C++ generator (csrc/tsdf_mesh.hip) so that tests can compare them:

  cube corners c = (x, y, z) bits (c & 1, c >> 1 & 1, c >> 2 & 1); a corner is INSIDE when its
  tsdf < 0; the 12 edges join corners differing in one bit; on each of the 6 faces, walked
  counter-clockwise as seen from outside the cube, every maximal run of inside corners gives
  one surface segment from the crossing where the walk leaves the run to the crossing where it
  entered it (so an ambiguous face keeps its two inside corners apart); segments chain into
  closed loops (each crossed edge starts one segment and ends one), and each loop is fanned
  into triangles from its first vertex.  The loops are taken in order of their smallest
  starting edge, and a loop starts at its smallest edge.
"""
from __future__ import annotations

CORNERS = [(c & 1, (c >> 1) & 1, (c >> 2) & 1) for c in range(8)]
# edges sorted by (axis, lower corner): index = axis * 4 + (the two other coordinate bits)
EDGES = []
for axis in range(3):
    for c in range(8):
        if not (c >> axis) & 1:
            EDGES.append((c, c | (1 << axis)))
EDGE_ID = {}
for i, (a, b) in enumerate(EDGES):
    EDGE_ID[(a, b)] = EDGE_ID[(b, a)] = i


def _faces():
    """6 faces as corner cycles, counter-clockwise seen from outside (outward normal)."""
    faces = []
    for axis in range(3):
        u, v = (axis + 1) % 3, (axis + 2) % 3  # (u, v, axis) right-handed
        for side in (0, 1):
            base = side << axis
            cyc = [base, base | (1 << u), base | (1 << u) | (1 << v), base | (1 << v)]
            if side == 0:  # outward normal is -axis: reverse to stay counter-clockwise
                cyc = cyc[::-1]
            faces.append(cyc)
    return faces


FACES = _faces()


def case_loops(cfg: int):
    inside = [(cfg >> c) & 1 for c in range(8)]
    seg = {}  # start edge -> end edge
    for cyc in FACES:
        n = 4
        if all(inside[c] for c in cyc) or not any(inside[c] for c in cyc):
            continue
        for i in range(n):
            a, b = cyc[i], cyc[(i + 1) % n]
            if inside[a] and not inside[b]:  # leaving a run at edge (a, b)
                # walk back to where the run was entered
                j = i
                while inside[cyc[(j - 1) % n]]:
                    j -= 1
                p, q = cyc[(j - 1) % n], cyc[j % n]  # entering edge (p outside, q inside)
                seg[EDGE_ID[(a, b)]] = EDGE_ID[(p, q)]
    loops = []
    left = dict(seg)
    while left:
        start = min(left)
        loop = [start]
        e = left.pop(start)
        while e != start:
            loop.append(e)
            e = left.pop(e)
        loops.append(loop)
    return loops


def triangles(cfg: int):
    tris = []
    for loop in case_loops(cfg):
        for i in range(1, len(loop) - 1):
            tris.append((loop[0], loop[i], loop[i + 1]))
    return tris


def table():
    """256 x 16 list of edge ids, -1 padded (at most 5 triangles per case)."""
    out = []
    for cfg in range(256):
        t = [e for tri in triangles(cfg) for e in tri]
        assert len(t) <= 15, (cfg, len(t))
        out.append(t + [-1] * (16 - len(t)))
    return out
