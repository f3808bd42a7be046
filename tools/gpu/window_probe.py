"""Where does the dense integrate's per-update cost depend on the timed window?  (VERDICT r03
weak #1: the driver's `--steps 20 --warmup 5` window, frames 40-199, costs 13 % more per updated
voxel than the 250-step window.)

Runs on the bench's own resident frames (bench.py's generator) and prints one JSON line per row:
  * "chunks":  frames 0..F-1 integrated in order as calls of `chunk` frames; per call the
    HIP-event kernel time per launch, V_f and ns per voxel update (the trajectory's own cost
    profile, no reset in between);
  * "driver":  reset, 5 warm-up batches, 20 timed batches (the driver's command), repeated;
  * "heated":  the same after a 200-batch run on another volume right before it (clock / power
    state effects, if any, show as a difference to "driver");
  * "late":    reset, W warm-up batches, 20 timed batches for later W (the trajectory's effect).

    PYTHONPATH=union-thesis-slam_amd python tools/gpu/window_probe.py [chunk]
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))
from tsdf_amd import grid_fusion, scene  # noqa: E402

B = 8


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 160
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
    dptr, cptr = depth.data_ptr(), rgb.data_ptr()
    ds, cs = 480 * 640 * 2, 480 * 640 * 3
    vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)

    def run(v, start, n, prof):
        v.set_profiling(prof)
        v.stats(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = start
        while n > 0:
            s %= F
            m = min(n, F - s)
            v.integrate_batch(dptr + s * ds, cptr + s * cs, K, Tinv[s:s + m], hw=(480, 640), device_ptrs=True,
                              sync=False)
            s += m
            n -= m
        v.sync()
        dt = time.perf_counter() - t0
        st = v.stats()
        return dt, st

    def row(kind, start, n, dt, st, **kw):
        L = max(1, st["kernel_launches"])
        us = 1e3 * st["kernel_ms"] / L
        r = {"kind": kind, "first_frame": start, "frames": n, "fps_wall": round(n / dt, 1),
             "kernel_us_per_launch": round(us, 2), "launches": st["kernel_launches"],
             "vf_mean": round(st["voxel_updates"] / n), "ns_per_update_kernel":
             round(1e6 * st["kernel_ms"] / max(1, st["voxel_updates"]), 5),
             "visited_per_frame": round(st["bricks_visited"] / n), "touched_per_frame": round(st["bricks_touched"] / n)}
        r.update(kw)
        print(json.dumps(r), flush=True)

    # the trajectory's cost profile: chunks in order, no reset
    vol.reset()
    for s0 in range(0, F, chunk):
        dt, st = run(vol, s0, chunk, True)
        row("chunks", s0, chunk, dt, st)
    # the driver's window, repeated
    for rep in range(3):
        vol.reset()
        run(vol, 0, 5 * B, False)
        dt, st = run(vol, 5 * B, 20 * B, True)
        row("driver", 5 * B, 20 * B, dt, st, rep=rep)
    # heated: a long run on another volume right before
    other = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)
    for rep in range(2):
        vol.reset()
        run(other, 0, 200 * B, False)
        run(vol, 0, 5 * B, False)
        dt, st = run(vol, 5 * B, 20 * B, True)
        row("heated", 5 * B, 20 * B, dt, st, rep=rep)
    other.close()
    # the 250-step default window, and later 20-batch windows
    vol.reset()
    run(vol, 0, 12 * B, False)
    dt, st = run(vol, 12 * B, 250 * B, True)
    row("default250", 12 * B, 250 * B, dt, st)
    for w in (25, 50, 100):
        vol.reset()
        run(vol, 0, w * B, False)
        dt, st = run(vol, w * B, 20 * B, True)
        row("late", w * B, 20 * B, dt, st)
    # the same window with the volume continued (no reset, so the first 40 frames are long past)
    vol.reset()
    run(vol, 0, 1000, False)
    dt, st = run(vol, 5 * B, 20 * B, True)
    row("revisit", 5 * B, 20 * B, dt, st)
    vol.close()


if __name__ == "__main__":
    main()
