"""Diagnostic: a mapped (VMM) block pool through synchronous and asynchronous growth at 512^3;
prints pool_mapped / capacity after each call and the library's last error message."""
import sys

import numpy as np

sys.path.insert(0, "union-thesis-slam_amd")
sys.path.insert(0, "tests")
from tsdf_amd import _ffi, hash_fusion, scene  # noqa: E402

poses = scene.trajectory(40, seed=0, start=100)
d, c = scene.render(poses, scene.make_spheres(0), seed=0, start=100)
d, c = d.numpy(), c.numpy()
K = scene.intrinsics()
Tinv = np.linalg.inv(poses)
h = hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), 0.02, 1 << 16, max_blocks=1 << 12)
last = lambda: _ffi.load().tsdf_last_error().decode()
for lo, hi, sync in ((0, 8, True), (8, 16, True), (16, 40, False)):
    h.integrate_batch(d[lo:hi], c[lo:hi], K, Tinv[lo:hi], sync=sync)
    h.sync()
    i = h.info()
    print(lo, hi, sync, "mapped", i["pool_mapped"], "cap", i["pool_capacity"], "top", i["blocks_in_pool"],
          "err:", last(), flush=True)
