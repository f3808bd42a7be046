#!/usr/bin/env python3
"""Host-side issue cost of the dense integrate: wall time of the asynchronous integrate_batch
calls (they return once every batch is enqueued) vs the time until the GPU has finished, for a
shard of an N-way cyclic split.  python tools/host_issue.py [--only 8:0] [--frames 400]"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="8:0")
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    import torch
    from tsdf_amd import grid_fusion, scene
    dev = torch.device("cuda", 0)
    F = a.frames
    poses = scene.trajectory(F, seed=0)
    sph = scene.make_spheres(0)
    depth = torch.empty((F, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((F, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, F, 50):
        d, c = scene.render(poses[s:s + 50], sph, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    K = scene.intrinsics()
    world, r = (int(x) for x in a.only.split(":"))
    with contextlib.redirect_stdout(sys.stderr):
        vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02, shard=(r, world))
    out = {}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=False)
        t1 = time.perf_counter()
        vol.sync()
        t2 = time.perf_counter()
        out = {"only": a.only, "batches": (F + 7) // 8, "issue_us_per_batch": round((t1 - t0) / ((F + 7) // 8) * 1e6, 2),
               "total_us_per_batch": round((t2 - t0) / ((F + 7) // 8) * 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
