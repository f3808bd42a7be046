"""The z-half protocol's events in the bench's hash window (diagnostic build: tools/build_variant.sh
hdiag "-DTSDF_HASH_DIAG", run with TSDF_HIP_LIB=abtest/libhdiag.so): a fresh 2^22 table, 5
synchronous batches, then the 20 timed batches (inserting), then the same 20 again (every block
exists).  Per window: items, z-low re-lookups (and how many found the block), z-high waits at item
start and their sleep iterations, end claims (inserts), end waits for the claimer and their sleep
iterations, and the launches' average time.  One JSON line per window.

    PYTHONPATH=union-thesis-slam_amd TSDF_HIP_LIB=abtest/libhdiag.so python tools/gpu/hash_diag.py
"""
import contextlib
import ctypes
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "union-thesis-slam_amd"))
from tsdf_amd import _ffi, hash_fusion, scene  # noqa: E402

NAMES = ["items", "relookups", "relookups_found", "zhigh_start_waits", "zhigh_start_spins", "claims",
         "end_waits", "end_wait_spins"]


def main():
    dev = torch.device("cuda", 0)
    F = 1000
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
    ds, cs = depth[0].numel() * 2, rgb[0].numel()
    lib = _ffi.load()
    fn = lib.tsdf_diag_hash_counts
    fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros(24, np.uint64)
    with contextlib.redirect_stdout(io.StringIO()):
        ht = hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), 0.02, 1 << 22, max_blocks=1 << 15)
    B = ht.frames_per_launch()
    ht.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv[:5 * B], hw=(480, 640), device_ptrs=True)
    fn(buf.ctypes.data)
    for label in ("driver window, fresh table (inserting)", "the same window again (every block exists)"):
        ht.set_profiling(True)
        ht.stats(reset=True)
        ht.integrate_batch(depth.data_ptr() + 5 * B * ds, rgb.data_ptr() + 5 * B * cs, K, Tinv[5 * B:25 * B],
                           hw=(480, 640), device_ptrs=True, sync=False)
        ht.sync()
        st = ht.stats()
        fn(buf.ctypes.data)
        out = {"window": label, "kernel_avg_us": round(1e3 * st["kernel_ms"] / max(1, st["kernel_launches"]), 1),
               "launches": st["kernel_launches"], "blocks_allocated": st["blocks_allocated"]}
        out.update({k: int(v) for k, v in zip(NAMES, buf)})
        for c, name in enumerate(("found_by_cull", "missing_not_updated", "claimer", "partner_waited",
                                  "found_after_start_lookup")):
            n, ticks = int(buf[8 + 2 * c]), int(buf[9 + 2 * c])
            out[name] = {"items": n, "mean_us": round(ticks / 100.0 / max(1, n), 2)}
        print(json.dumps(out), flush=True)
    ht.close()


if __name__ == "__main__":
    main()
