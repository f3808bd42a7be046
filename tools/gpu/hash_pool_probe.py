"""Does the hash's driver window pay for its pool growth?  The bench's hash leg (fresh 2^22-slot
table, 5 synchronous warm-up batches, 20 timed asynchronous batches) with the bench's initial pool
(2^15 blocks, grown by mapping during the window) against a pool mapped for every brick of the
volume from the start (2^18: no growth), each three times, after a clock warm-up.

    PYTHONPATH=union-thesis-slam_amd python tools/gpu/hash_pool_probe.py [premapped]

(premapped: the second configuration only -- with TSDF_HASH_VMM=0, plain allocations against the
reserved-and-mapped ranges, the same pool size)
"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "union-thesis-slam_amd"))
from tsdf_amd import grid_fusion, hash_fusion, scene  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    F = 400
    poses = scene.trajectory(F, seed=0, radius_frac=scene.BENCH_RING)
    sph = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((F, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((F, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, F, 50):
        d, c = scene.render(poses[s:s + 50], sph, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    K = scene.intrinsics()
    bnds = np.array([[0.0, 10.24]] * 3)
    ds, cs = depth[0].numel() * 2, rgb[0].numel()
    with contextlib.redirect_stdout(io.StringIO()):
        vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02)
    t_end = time.perf_counter() + 0.3  # clock warm-up
    while time.perf_counter() < t_end:
        vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv[:160], hw=(480, 640), device_ptrs=True)
    vol.close()
    out = {}
    cfgs = (("pool_2^15_grown", 1 << 15), ("pool_2^18_premapped", 1 << 18))
    if sys.argv[1:] == ["premapped"]:
        cfgs = cfgs[1:]
    tag = "vmm" if os.environ.get("TSDF_HASH_VMM", "1") != "0" else "plain"
    for name, mb in cfgs:
        name = f"{name}_{tag}"
        rows = []
        for _ in range(3):
            with contextlib.redirect_stdout(io.StringIO()):
                ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=mb)
            ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv[:40], hw=(480, 640), device_ptrs=True)
            ht.set_profiling(True)
            ht.stats(reset=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ht.integrate_batch(depth.data_ptr() + 40 * ds, rgb.data_ptr() + 40 * cs, K, Tinv[40:200], hw=(480, 640),
                               device_ptrs=True, sync=False)
            ht.sync()
            dt = time.perf_counter() - t0
            st = ht.stats()
            rows.append({"fps": round(160 / dt, 1), "kernel_avg_us": round(1e3 * st["kernel_ms"] / st["kernel_launches"], 2),
                         "allocated": st["blocks_allocated"], "skipped": st["bricks_skipped"],
                         "pool_capacity": ht.info()["pool_capacity"]})
            ht.close()
        out[name] = rows
        print(json.dumps({name: rows}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
