#!/usr/bin/env python3
"""Hash extraction on the device (HashTable.get_mesh / get_point_cloud, hash_fusion.py:465-507):
the bench frames into a voxel hash at 512^3 @ 2 cm and 1024^3 @ 1 cm, then
  * tsdf_hash_to_dense: the live blocks densified into a dense handle on the device,
  * the dense handle's marching cubes,
  * for comparison, the round-2 path: get_state (device -> host) + set_state (host -> device).
Prints one JSON object.   PYTHONPATH=union-thesis-slam_amd python tools/gpu/hash_extract_time.py"""
import contextlib
import ctypes
import io
import json
import sys
import time

import numpy as np
import torch

from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene


def main(frames=400):
    dev = torch.device("cuda", 0)
    poses = scene.trajectory(frames, seed=0, radius_frac=scene.BENCH_RING)
    sph = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((frames, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((frames, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, frames, 50):
        d, c = scene.render(poses[s:s + 50], sph, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    K = scene.intrinsics()
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    out = {"frames": frames}
    for vs in (0.02, 0.01):
        bnds = np.array([[0.0, 10.24]] * 3)
        with contextlib.redirect_stdout(io.StringIO()):
            ht = hash_fusion.HashTable(bnds.copy(), vs, 1 << 22, max_blocks=1 << 16)
        ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True)
        r = {"blocks_live": ht.info()["used"]}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            grid = ht._as_grid()
        r["to_dense_handle_s"] = round(time.perf_counter() - t0, 4)  # includes the dense handle's allocation
        t0 = time.perf_counter()
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        _ffi.call("tsdf_dense_extract_mesh", grid._h, ctypes.byref(nv), ctypes.byref(nt))
        r["marching_cubes_s"] = round(time.perf_counter() - t0, 4)
        r["triangles"] = nt.value
        t0 = time.perf_counter()
        t, w, c = ht.get_state()
        grid.set_state(t, w, c)
        r["host_round_trip_s"] = round(time.perf_counter() - t0, 4)
        r["dense_extent_bytes"] = int(3 * t.nbytes)
        del t, w, c
        grid.close()
        ht.close()
        torch.cuda.empty_cache()
        out[f"{int(round(10.24 / vs))}^3"] = r
        print(json.dumps(r), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
