"""Where the time of an eighth-shard launch goes: per integrate workgroup of the last fused launch
of a call, its start, end and list items (diagnostic build: tools/build_variant.sh wgt
"-DTSDF_WG_TIMES", run with TSDF_HIP_LIB=abtest/libwgt.so).  Bench workload (scaling_sim's), one
GPU and rank 0 of 2 / 4 / 8 cyclic column shards.  Prints one JSON line per configuration."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, scene  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    F = 200
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
    lib = _ffi.load()
    fn = lib.tsdf_diag_wg_times
    fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros((3, 8192), np.uint64)
    for world in (1, 2, 4, 8):
        vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(0, world))
        rows = []
        for start in range(0, 192, 8):
            vol.integrate_batch(depth.data_ptr() + start * ds, rgb.data_ptr() + start * cs, K, Tinv[start:start + 8],
                                hw=(480, 640), device_ptrs=True)
            if start < 48:
                continue
            fn(buf.ctypes.data)
            n = int(np.count_nonzero(buf[1]))
            t0 = buf[0, :n].astype(np.int64)
            t1 = buf[1, :n].astype(np.int64)
            it = buf[2, :n].astype(np.int64)
            base = t0.min()
            s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # us
            rows.append([e.max(), np.median(e), np.percentile(e, 10), s.max(), (e - s).mean(), it.mean(), it.min(), it.max()])
        r = np.array(rows).mean(axis=0)
        if os.environ.get("WG_DUMP") and world in (1, 8):
            busy = (t1 - t0) / 100.0
            by_xcd = [round(float(busy[x::8].mean()), 1) for x in range(8)]
            pair = busy[:256] - busy[256:512] if n >= 512 else busy[:0]
            print(json.dumps({"world": world, "busy_by_xcd": by_xcd,
                              "busy_first_half": round(float(busy[:256].mean()), 1),
                              "busy_second_half": round(float(busy[256:].mean()), 1),
                              "items_corr": round(float(np.corrcoef(busy, it)[0, 1]), 3),
                              "pair_diff_std": round(float(pair.std()), 1) if len(pair) else None,
                              "busy_sorted_deciles": [round(float(x), 1) for x in np.percentile(busy, range(0, 101, 10))],
                              "busy_first32": [round(float(x), 1) for x in busy[:32]]}), flush=True)
        print(json.dumps({"world": world, "wgs": n, "span_us": round(r[0], 2), "end_median_us": round(r[1], 2),
                          "end_p10_us": round(r[2], 2), "last_start_us": round(r[3], 2),
                          "wg_busy_mean_us": round(r[4], 2), "items_mean": round(r[5], 1),
                          "items_min": int(r[6]), "items_max": int(r[7])}), flush=True)
        del vol


if __name__ == "__main__":
    main()
