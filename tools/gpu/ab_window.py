"""A/B probe of one library build (TSDF_HIP_LIB selects it) at the driver's own window: a fresh
volume, 5 untimed batches, 20 timed batches (bench.py --steps 20 --warmup 5), repeated; dense and
hash; plus the 250-step default window once, and frames 160-799 of a fresh volume (the same
frames whatever the build's frames per launch).  One JSON line.

    PYTHONPATH=union-thesis-slam_amd python tools/gpu/ab_window.py [reps] [name]
"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene  # noqa: E402

def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    name = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(_ffi.LIB_PATH)
    F = 1000
    dev = torch.device("cuda", 0)
    poses = scene.trajectory(F, seed=0, radius_frac=scene.BENCH_RING)
    spheres = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((F, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((F, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, F, 50):
        d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    K = scene.intrinsics()
    torch.cuda.synchronize()
    dkind = None
    if os.environ.get("AB_DEPTH") == "f64":  # the same frames as f64 metres (the integrate's DK = 1 path)
        depth = (depth.to(torch.int32) & 0xFFFF).to(torch.float64) / 1000.0
        dkind = _ffi.DEPTH_F64_M
        name += "_f64"
    dptr, cptr = depth.data_ptr(), rgb.data_ptr()
    ds, cs = 480 * 640 * depth.element_size(), 480 * 640 * 3

    def run(v, start, n, prof, sync=True):
        v.set_profiling(prof)
        v.stats(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s, left = start, n
        while left > 0:  # the frames cycle, as in bench.py
            s %= F
            m = min(left, F - s)
            v.integrate_batch(dptr + s * ds, cptr + s * cs, K, Tinv[s:s + m], hw=(480, 640), device_ptrs=True,
                              sync=sync, depth_kind=dkind)
            s += m
            left -= m
        v.sync()
        dt = time.perf_counter() - t0
        st = v.stats()
        return n / dt, 1e3 * st["kernel_ms"] / max(1, st["kernel_launches"]), (st["voxel_updates"], st["bricks_visited"])

    out = {"lib": name, "build_id": _ffi.build_id()}
    bnds = np.array([[0.0, 10.24]] * 3)
    vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02)
    B = vol.frames_per_launch()  # a step = one launch's frames, as in bench.py
    out["frames_per_launch"] = B
    rows = []
    for _ in range(reps):
        vol.reset()
        run(vol, 0, 5 * B, False, sync=False)
        rows.append(run(vol, 5 * B, 20 * B, True, sync=False))
    out["dense_driver_fps"] = round(statistics.median(r[0] for r in rows), 1)
    out["dense_driver_us"] = round(statistics.median(r[1] for r in rows), 2)
    out["dense_driver_all"] = [round(r[0]) for r in rows]
    vol.reset()
    run(vol, 0, 12 * B, False, sync=False)
    r = run(vol, 12 * B, 250 * B, True, sync=False)
    out["dense_250_fps"], out["dense_250_us"] = round(r[0], 1), round(r[1], 2)
    # the same frames whatever the launch size (160 untimed, then 640 timed: builds with 16- and
    # 32-frame launches compare on equal work), kernel time per frame
    rows = []
    for _ in range(reps):
        vol.reset()
        run(vol, 0, 160, False, sync=False)
        f, us, cnt = run(vol, 160, 640, True, sync=False)
        rows.append((f, us / B))
    out["dense_fixed_updates_visited"] = cnt  # (the cull's kept bricks: a check of the pyramid)
    out["dense_fixed_fps"] = round(statistics.median(r[0] for r in rows), 1)
    out["dense_fixed_us_per_frame"] = round(statistics.median(r[1] for r in rows), 3)
    vol.close()
    rows = []
    for _ in range(reps):
        ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=1 << 15)
        run(ht, 0, 5 * B, False, sync=True)
        rows.append(run(ht, 5 * B, 20 * B, True, sync=False))
        skipped = ht.stats()["bricks_skipped"]
        ht.close()
        if skipped:
            raise RuntimeError(f"hash skipped {skipped} bricks")
    out["hash_driver_fps"] = round(statistics.median(r[0] for r in rows), 1)
    out["hash_driver_us"] = round(statistics.median(r[1] for r in rows), 2)
    out["hash_driver_all"] = [round(r[0]) for r in rows]
    ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=1 << 15)
    run(ht, 0, 12 * B, False, sync=True)
    r = run(ht, 12 * B, 250 * B, True, sync=False)
    out["hash_250_fps"], out["hash_250_us"] = round(r[0], 1), round(r[1], 2)
    ht.close()
    rows = []
    for _ in range(reps):
        ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=1 << 15)
        run(ht, 0, 160, False, sync=True)
        f, us, _ = run(ht, 160, 640, True, sync=False)
        rows.append((f, us / B))
        ht.close()
    out["hash_fixed_fps"] = round(statistics.median(r[0] for r in rows), 1)
    out["hash_fixed_us_per_frame"] = round(statistics.median(r[1] for r in rows), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
