#!/usr/bin/env python3
"""Voxel-hash load-factor sweep (BASELINE config[2]): the bench's synthetic frames into the 512^3
@ 2 cm extent through tables of 2^18 .. 2^22 slots (8^3 blocks), one GPU.  The live block count
is fixed by the scene, so the table size sets the load factor.  Prints one JSON object:
per capacity frames/s, Mvoxel-updates/s, load factor, mean/max probe distance, displaced keys.

  python tools/hash_sweep.py [--steps 1000] [--warmup 100]
"""
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
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--log2", default="18,19,20,21,22")
    a = ap.parse_args()
    import torch
    from tsdf_amd import hash_fusion, scene
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
    dstride, cstride = depth[0].numel() * 2, rgb[0].numel()

    def run(ht, start, count):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = start
        while count > 0:
            b = s % F
            n = min(count, F - b)
            ht.integrate_batch(depth.data_ptr() + b * dstride, rgb.data_ptr() + b * cstride, K,
                               Tinv[b:b + n], hw=(480, 640), device_ptrs=True, sync=False)
            s += n
            count -= n
        ht.sync()
        return time.perf_counter() - t0

    out = []
    nb = 64 ** 3
    for lg in [int(x) for x in a.log2.split(",")]:
        with contextlib.redirect_stdout(sys.stderr):
            ht = hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), 0.02, 1 << lg, max_blocks=nb)
        run(ht, 0, a.warmup)
        ht.stats(reset=True)
        dt = run(ht, a.warmup, a.steps)
        st, info = ht.stats(), ht.info()
        if st["bricks_skipped"]:
            raise RuntimeError(f"2^{lg}: table overflowed")
        r = {"capacity": 1 << lg, "load_factor": round(info["used"] / info["capacity"], 4),
             "frames_per_s": round(a.steps / dt, 1),
             "mvox_updates_per_s": round(st["voxel_updates"] / dt / 1e6, 1),
             "mean_probe": round(st["probe_steps"] / max(1, st["lookups"]), 4),
             "max_probe": int(st["probe_max"]), "displaced": int(info["displaced"]),
             "blocks_live": int(info["used"])}
        print(json.dumps(r), file=sys.stderr, flush=True)
        out.append(r)
        del ht
        torch.cuda.empty_cache()
    print(json.dumps({"sweep": out, "steps": a.steps, "volume": "512^3 @ 2 cm extent, 8^3 blocks"}))


if __name__ == "__main__":
    main()
