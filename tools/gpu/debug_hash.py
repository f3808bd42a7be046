"""Debug: hash vs dense after frames 0 and 1 (lounge c1)."""
import sys, os
sys.path[:0] = ["union-thesis-slam_amd", "oracle", "tests"]
import numpy as np
from conftest import load_lounge, lounge_intrinsics
from tsdf_amd import grid_fusion, hash_fusion
C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]
K = lounge_intrinsics()
g = grid_fusion.TSDFVolume(np.array(C1), 0.04)
h = hash_fusion.HashTable(np.array(C1), 0.04, 1000000)
for f in range(3):
    _, depth, rgb, pose = load_lounge(f)
    g.integrate(rgb, depth, K, pose)
    h.integrate(rgb, depth, K, pose)
    G = g.get_state(); H = h.get_state()
    st = h.stats(); inf = h.info()
    print("frame", f, "dense entries", int((G[1] > 0).sum()), "hash entries", int((H[1] > 0).sum()),
          "alloc", st["blocks_allocated"], "lookups", st["lookups"], "info", inf)
    bad = np.flatnonzero((G[1] != H[1]).reshape(-1))
    print("  weight mismatches", len(bad), "tsdf mism", int((G[0] != H[0]).sum()), "color mism", int((G[2] != H[2]).sum()))
    if len(bad):
        pos = np.stack(np.unravel_index(bad[:10], G[1].shape), 1)
        print("  first", pos.tolist(), G[1].reshape(-1)[bad[:10]], H[1].reshape(-1)[bad[:10]])
        blocks = np.unique(np.stack(np.unravel_index(bad, G[1].shape), 1) // 8, axis=0)
        print("  bad blocks", len(blocks))
