"""Throughput over a long sequence (SURVEY §8(d) C4 per GPU: the bench trajectory continued for
10k frames into one 512^3 @ 2 cm volume): frames/s per chunk of 1000 frames and the largest
weight, to see where weights pass the fast path's reciprocal-table limit (csrc/tsdf_device.h
small_int) and what that costs.

    python tools/gpu/long_run.py [frames] [chunk]
"""
import json
import sys
import time

import numpy as np
import torch

from tsdf_amd import grid_fusion, scene


def main():
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    dev = torch.device("cuda", 0)
    spheres = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    K = scene.intrinsics()
    vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)
    depth = torch.empty((chunk, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((chunk, 480, 640, 3), dtype=torch.uint8, device=dev)
    out = []
    for s0 in range(0, total, chunk):
        poses = scene.trajectory(chunk, seed=0, start=s0, radius_frac=scene.BENCH_RING)
        for s in range(0, chunk, 50):
            d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=s0 + s, device=dev, depth_dtype=torch.int16)
            depth[s:s + len(d)] = d
            rgb[s:s + len(c)] = c
        torch.cuda.synchronize()
        vol.stats(reset=True)
        t0 = time.perf_counter()
        vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, np.linalg.inv(poses), hw=(480, 640),
                            device_ptrs=True, sync=False)
        vol.sync()
        dt = time.perf_counter() - t0
        st = vol.stats()
        wmax = float(vol.get_rows(np.arange(0, 512, 16))[1].max())
        row = {"first_frame": s0, "frames": chunk, "fps": round(chunk / dt, 1),
               "mvox_per_s": round(st["voxel_updates"] / dt / 1e6, 1), "max_weight_sampled_rows": wmax}
        out.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"long_run": out}))


if __name__ == "__main__":
    main()
