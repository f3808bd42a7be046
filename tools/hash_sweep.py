#!/usr/bin/env python3
"""Voxel-hash load-factor sweep (BASELINE config[2]): the bench's synthetic
frames into the 512^3 @ 2 cm extent (8^3 blocks) through tables whose capacity puts the final
load factor at 0.1 .. 0.9 (non-power-of-two capacities; floor-mod home slots like the
reference), one GPU.  The resize policy is lifted to 0.95 (TSDF_HASH_MAX_LOAD) so the table keeps
its size.  Per capacity: the insert pass (first pass over the frames, synchronous, every block
allocated there) and the steady pass (the same frames again: lookups only), frames/s, Mvoxel-updates/s,
mean / max probe distance, displaced keys.  Also the 1024^3 @ 1 cm extent's cull cost (same
frames, 2^22 buckets, 8x the bricks the cull walks).  Prints one JSON object.

  python tools/hash_sweep.py [--frames 400]
"""
import argparse
import contextlib
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--loads", default="0.1,0.25,0.5,0.6,0.7,0.75,0.8,0.85,0.9")
    a = ap.parse_args()
    os.environ["TSDF_HASH_MAX_LOAD"] = "0.95"
    import torch
    from tsdf_amd import hash_fusion, scene
    dev = torch.device("cuda", 0)
    F = a.frames
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

    def run(ht, sync=False):
        ht.stats(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv, hw=(480, 640), device_ptrs=True, sync=sync)
        ht.sync()
        dt = time.perf_counter() - t0
        st = ht.stats()
        if st["bricks_skipped"] and not sync:
            raise RuntimeError("bricks skipped")
        return dt, st

    def table(vs, cap, max_blocks):
        with contextlib.redirect_stdout(sys.stderr):
            return hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), vs, cap, max_blocks=max_blocks)

    # the scene's live block count at the end of one pass
    ht = table(0.02, 1 << 22, 64 ** 3)
    run(ht)
    live = ht.info()["used"]
    del ht
    torch.cuda.empty_cache()
    out = []
    for lf in [float(x) for x in a.loads.split(",")]:
        cap = int(math.ceil(live / lf))
        ht = table(0.02, cap, 64 ** 3)
        r = {"target_load": lf, "capacity": cap}
        # the insert pass is synchronous (the resize policy alone decides the table size: the
        # asynchronous growth headroom would resize it early); the steady pass is asynchronous
        for name, sync in (("insert_pass", True), ("steady_pass", False)):
            dt, st = run(ht, sync)
            info = ht.info()
            r[name] = {"frames_per_s": round(F / dt, 1), "mvox_updates_per_s": round(st["voxel_updates"] / dt / 1e6, 1),
                       "mean_probe": round(st["probe_steps"] / max(1, st["lookups"]), 3),
                       "max_probe": int(st["probe_max"]), "blocks_allocated": int(st["blocks_allocated"])}
        r.update({"load_factor": round(info["used"] / info["capacity"], 4), "displaced": int(info["displaced"]),
                  "blocks_live": int(info["used"]), "capacity_final": int(info["capacity"])})
        print(json.dumps(r), file=sys.stderr, flush=True)
        out.append(r)
        del ht
        torch.cuda.empty_cache()
    # 1024^3 @ 1 cm extent (config[4]'s): the cull walks 2^21 bricks per batch
    ext = {}
    for vs, nb in ((0.02, 64 ** 3), (0.01, 128 ** 3)):
        ht = table(vs, 1 << 22, min(nb, 1 << 20))
        run(ht)  # allocate
        ht.set_profiling(True)
        dt, st = run(ht)
        ext[f"{int(round(10.24 / vs))}^3"] = {
            "frames_per_s": round(F / dt, 1), "kernel_avg_us": round(1e3 * st["kernel_ms"] / max(1, st["kernel_launches"]), 1),
            "bricks_in_extent": nb, "bricks_visited_per_frame": round(st["bricks_visited"] / F),
            "voxel_updates_per_frame": round(st["voxel_updates"] / F), "blocks_live": int(ht.info()["used"])}
        print(json.dumps(ext), file=sys.stderr, flush=True)
        del ht
        torch.cuda.empty_cache()
    print(json.dumps({"sweep": out, "frames": F, "live_blocks": live, "extent_cost": ext,
                      "volume": "512^3 @ 2 cm extent, 8^3 blocks, bench ring frames"}))


if __name__ == "__main__":
    main()
