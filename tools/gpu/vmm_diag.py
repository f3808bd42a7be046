"""Which phase of an asynchronous / trimmed VMM hash run departs from the dense grid: runs the
trim test's trajectory in variants (sync only, async, async + trim, sync + trim) and prints the
first mismatching voxel count per variant.  Diagnostic only (GPU)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "union-thesis-slam_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
from test_dropin_gpu import BNDS, _synth  # noqa: E402
from tsdf_amd import grid_fusion, hash_fusion  # noqa: E402


def run(async_mid, trim, peek, n=64):
    d, c, poses = _synth(n, start=100)
    K = np.array([[585.0, 0, 320], [0, 585.0, 240], [0, 0, 1]])
    Tinv = np.linalg.inv(poses)
    h = hash_fusion.HashTable(np.array(BNDS), 0.02, 1 << 16, max_blocks=1 << 12)
    h.integrate_batch(d[:8], c[:8], K, Tinv[:8])
    h.integrate_batch(d[8:40], c[8:40], K, Tinv[8:40], sync=not async_mid)
    h.sync()
    i1 = h.info()
    g = grid_fusion.TSDFVolume(np.array(BNDS), 0.02)
    g.integrate_batch(d[:40], c[:40], K, Tinv[:40])
    bad40 = [int((a != b).sum()) for a, b in zip(g.get_state(), h.get_state())] if peek else None
    if trim:
        h.trim()
    i2 = h.info()
    h.integrate_batch(d[40:], c[40:], K, Tinv[40:])
    g.integrate_batch(d[40:], c[40:], K, Tinv[40:])
    gs, hs = g.get_state(), h.get_state()
    bad = [int((a != b).sum()) for a, b in zip(gs, hs)]
    for k, (a, b) in enumerate(zip(gs, hs)):
        idx = np.argwhere(a != b)
        if len(idx):
            bricks = np.unique(idx // 8, axis=0)
            i = tuple(idx[: 6].T)
            print(f"  array {k}: {len(bricks)} bricks, first {bricks[:4].tolist()}, expected {a[i]}, got {b[i]},"
                  f" weights {gs[1][i]} / {hs[1][i]}, got-value range {b[tuple(idx.T)].min()} .. {b[tuple(idx.T)].max()}",
                  flush=True)
    print(f"async={async_mid} trim={trim} peek={peek}: at 40 {bad40} end {bad} pool {i1['pool_capacity']} -> "
          f"{i2['pool_capacity']} -> {h.info()['pool_capacity']} mapped {i1['pool_mapped']} "
          f"used {h.info()['used']} stats {h.stats()}", flush=True)


if __name__ == "__main__":
    for a, t, p in [(False, True, False), (True, True, False)] * 3:
        run(a, t, p)
