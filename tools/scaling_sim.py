#!/usr/bin/env python3
"""Predict the N-GPU strong-scaling curve of the dense bench on ONE GPU: every rank's shard of
512^3 @ 2 cm is built and timed in turn on the same synthetic frames; the N-rank job time is the
max over its ranks (ranks never exchange data while integrating).  Compares contiguous slabs
with cyclic 8-voxel column shards.  --hash: the voxel hash's bucket-range shards
(BASELINE config[4]: 2^22 buckets; --extent 1024 puts the same room into a 1024^3 @ 1 cm extent),
with each rank's frames/s, Mvoxel-updates/s and HBM state bytes.

  python tools/scaling_sim.py [--steps 800] [--warmup 48] [--worlds 1,2,4,8]
  python tools/scaling_sim.py --hash [--extent 512|1024] [--only 8:5]
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
    ap.add_argument("--hash", action="store_true", help="bucket-range hash shards instead of dense columns")
    ap.add_argument("--extent", type=int, default=512, help="hash: 512 (2 cm) or 1024 (1 cm) voxels per axis")
    ap.add_argument("--kernel-time", action="store_true", help="also time the integrate launches (HIP events)")
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
    if a.hash:
        return hash_shards(a, timed, bnds)
    if a.only:
        world, r = (int(x) for x in a.only.split(":"))
        with contextlib.redirect_stdout(sys.stderr):
            vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(r, world))
        timed(vol, 0, a.warmup)
        vol.set_profiling(a.kernel_time)
        vol.stats(reset=True)
        t = timed(vol, a.warmup, a.steps)
        st = vol.stats()
        r = {"only": a.only, "fps": round(a.steps / t, 1), "stats": st}
        if a.kernel_time:
            r["kernel_avg_us"] = round(1e3 * st["kernel_ms"] / max(1, st["kernel_launches"]), 2)
            r["launches"] = st["kernel_launches"]
        print(json.dumps(r, default=float))
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
    from tsdf_amd import _ffi
    out["build_id"] = _ffi.build_id()
    print(json.dumps(out))


def hash_shards(a, timed, bnds):
    """Bucket-range shards of the voxel hash (shard r of N owns the blocks whose home slot is in
    [r S / N, (r+1) S / N), S = 2^22): each rank's shard timed in turn on the same frames."""
    import torch
    from tsdf_amd import hash_fusion
    vs = 10.24 / a.extent
    per_block = 3 * 4 * 512 + 64 + 4
    out = {"extent": f"{a.extent}^3 @ {vs * 100:g} cm", "buckets": 1 << 22,
           "dense_shard_bytes_note": "dense grid of the same extent / N: 12 B per voxel"}
    worlds = [int(a.only.split(":")[0])] if a.only else [int(w) for w in a.worlds.split(",")]
    for world in worlds:
        ranks = [int(a.only.split(":")[1])] if a.only else range(world)
        res = []
        for r in ranks:
            with contextlib.redirect_stdout(sys.stderr):
                ht = hash_fusion.HashTable(bnds.copy(), vs, 1 << 22, shard=r, n_shards=world,
                                           max_blocks=1 << 15)
            timed(ht, 0, a.warmup)
            ht.set_profiling(a.kernel_time)
            ht.stats(reset=True)
            t = timed(ht, a.warmup, a.steps)
            st = ht.stats()
            ht.stats(reset=True)
            t2 = timed(ht, a.warmup, a.steps)  # the same window again: every block exists
            st2 = ht.stats()
            ht.trim()  # the pool at its live blocks (the run's growth headroom handed back)
            info = ht.info()
            state = info["slots"] * 12 + info["pool_capacity"] * per_block
            res.append({"rank": r, "fps": round(a.steps / t, 1),
                        "mvox_updates_per_s": round(st["voxel_updates"] / t / 1e6, 1),
                        "blocks_live": info["used"], "pool_capacity": info["pool_capacity"],
                        "hbm_state_bytes": state,
                        "dense_shard_bytes": 12 * a.extent ** 3 // world,
                        "bricks_skipped": st["bricks_skipped"], "blocks_allocated": st["blocks_allocated"]})
            res[-1]["no_alloc_repeat"] = {"fps": round(a.steps / t2, 1), "blocks_allocated": st2["blocks_allocated"]}
            if a.kernel_time:
                res[-1]["kernel_avg_us"] = round(1e3 * st["kernel_ms"] / max(1, st["kernel_launches"]), 2)
                res[-1]["launches"] = st["kernel_launches"]
                res[-1]["no_alloc_repeat"]["kernel_avg_us"] = round(1e3 * st2["kernel_ms"] / max(1, st2["kernel_launches"]), 2)
            print(json.dumps(res[-1]), file=sys.stderr, flush=True)
            ht.close()
            del ht
            torch.cuda.empty_cache()
        t_max = min(x["fps"] for x in res)
        out[f"hash{world}"] = {"fps": t_max, "ranks": res}
    if "hash1" in out:
        base = out["hash1"]["fps"]
        for k, v in out.items():
            if k.startswith("hash"):
                v["predicted_efficiency"] = round(v["fps"] / (int(k[4:]) * base), 3)
    from tsdf_amd import _ffi
    out["build_id"] = _ffi.build_id()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
