#!/usr/bin/env python3
"""Predict the N-GPU strong-scaling curve of the dense bench on ONE GPU: every rank's shard of
512^3 @ 2 cm is built and timed in turn on the same synthetic frames; the N-rank job time is the
max over its ranks (ranks never exchange data while integrating).  Compares contiguous slabs
with cyclic 8-voxel column shards.

  python tools/scaling_sim.py [--steps 800] [--warmup 48] [--worlds 1,2,4,8]
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
    ap.add_argument("--steps", type=int, default=800, help="timed frames")
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--only", default=None, help="W:R -- time only rank R of world W (for profiling)")
    a = ap.parse_args()
    import torch
    from tsdf_amd import grid_fusion, scene, sharding
    dev = torch.device("cuda", 0)
    F = a.frames
    poses = scene.trajectory(F, seed=0, radius_frac=scene.BENCH_RING)  # the bench's workload
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
    X = 512
    dstride, cstride = depth[0].numel() * 2, rgb[0].numel()

    def timed(vol, start, count):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = start
        while count > 0:
            b = s % F
            n = min(count, F - b)
            vol.integrate_batch(depth.data_ptr() + b * dstride, rgb.data_ptr() + b * cstride, K,
                                Tinv[b:b + n], hw=(480, 640), device_ptrs=True, sync=False)
            s += n
            count -= n
        vol.sync()
        return time.perf_counter() - t0

    out = {}
    if a.only:
        world, r = (int(x) for x in a.only.split(":"))
        with contextlib.redirect_stdout(sys.stderr):
            vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(r, world))
        timed(vol, 0, a.warmup)
        vol.stats(reset=True)
        t = timed(vol, a.warmup, a.steps)
        print(json.dumps({"only": a.only, "fps": round(a.steps / t, 1), "stats": vol.stats()}, default=float))
        return
    for world in [int(w) for w in a.worlds.split(",")]:
        for mode in ("slab", "cyclic"):
            if world == 1 and mode == "cyclic":
                continue
            times, vox = [], []
            for r in range(world):
                with contextlib.redirect_stdout(sys.stderr):
                    kw = {"shard": (r, world)} if mode == "cyclic" else {"slab": sharding.slab(r, world, X)}
                    vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, **kw)
                timed(vol, 0, a.warmup)
                vol.stats(reset=True)
                times.append(timed(vol, a.warmup, a.steps))
                vox.append(vol.stats()["voxel_updates"])
                del vol
                torch.cuda.empty_cache()
            t = max(times)
            out[f"{mode}{world}"] = {"fps": round(a.steps / t, 1), "rank_fps": [round(a.steps / x, 1) for x in times],
                                     "max_over_mean": round(t / np.mean(times), 3),
                                     "vox_max_over_mean": round(max(vox) / np.mean(vox), 3)}
            print(f"{mode}{world}: {json.dumps(out[f'{mode}{world}'])}", file=sys.stderr, flush=True)
    base = out["slab1"]["fps"]
    for k, v in out.items():
        n = int(k.lstrip("slabcyclic"))
        v["predicted_efficiency"] = round(v["fps"] / (n * base), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
