"""Host timestamps of the per-frame drop-in (the reference's one-integrate()-per-frame loop,
grid_demo1.py:76-87 / hash_demo1.py:114-125): the duration of every integrate() call, split into
the calls that only copy a frame into the deferred batch and the calls that also launch it
(every TSDF_DEFER_FRAMES-th), for the dense volume and the hash table on the same frames.

    PYTHONPATH=union-thesis-slam_amd python tools/gpu/dropin_trace.py [frames] [passes] [dense,hash] [grains]

grains: comma-separated TSDF_DEFER_DMA_FRAMES values to compare (each handle reads it at create;
8 = the whole batch's DMA at the flush, round 4's behaviour).

Run it under `rocprofv3 --kernel-trace --stats` as well to set the GPU time per launched batch
beside the host's time per batch.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene  # noqa: E402

HOST_PARTS = ["deferred_flushes_us", "report_wait_us", "prepare_batch_us", "launches_us", "call_end_us",
              "flushes", "unused6", "other_flushes_us"]


def stats(us):
    a = np.asarray(us, dtype=np.float64)
    if a.size == 0:
        return None
    return {"n": int(a.size), "mean_us": round(float(a.mean()), 1), "p50_us": round(float(np.median(a)), 1),
            "p90_us": round(float(np.percentile(a, 90)), 1), "max_us": round(float(a.max()), 1)}


def main():
    nd = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    which = sys.argv[3].split(",") if len(sys.argv) > 3 else ["dense", "hash"]
    grains = sys.argv[4].split(",") if len(sys.argv) > 4 else [None]
    per = int(os.environ.get("TSDF_DEFER_FRAMES", "8"))
    poses = scene.trajectory(nd, seed=0, radius_frac=scene.BENCH_RING)
    d, c = scene.render(poses, scene.make_spheres(0, ring_frac=scene.BENCH_RING), seed=0,
                        device=torch.device("cuda", 0), depth_dtype=torch.int16)
    d64 = d.cpu().numpy().view(np.uint16).astype(np.float64) / 1000.0
    ch = c.cpu().numpy()
    K = scene.intrinsics()
    makers = {"dense": lambda: grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02),
              "hash": lambda: hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), 0.02, 1 << 22,
                                                    max_blocks=1 << 15)}
    out = {"frames": nd, "passes": passes, "defer_frames": per}
    # (a -DTSDF_HOST_TIMES build: the hash flush's host time by part, tsdf_diag_host_times)
    lib = _ffi.load()
    host_times = getattr(lib, "tsdf_diag_host_times", None) if hasattr(lib, "tsdf_diag_host_times") else None
    buf = (ctypes.c_double * 8)()
    for grain, name in [(g, w) for g in grains for w in which]:
        if grain is not None:
            os.environ["TSDF_DEFER_DMA_FRAMES"] = grain
        v = makers[name]()
        v.integrate(ch[0], d64[0], K, poses[0])
        v.sync()
        res = []
        for p in range(passes):
            if host_times is not None:
                host_times(buf)
            push, launch = [], []
            t_start = time.perf_counter()
            for i in range(nd):
                t0 = time.perf_counter()
                v.integrate(ch[i], d64[i], K, poses[i])
                dt = (time.perf_counter() - t0) * 1e6
                (launch if (i + 1) % per == 0 else push).append(dt)
            t1 = time.perf_counter()
            v.sync()
            t_end = time.perf_counter()
            res.append({"pass": p, "frames_per_s": round(nd / (t_end - t_start), 1),
                        "final_sync_us": round((t_end - t1) * 1e6, 1), "copy_calls": stats(push),
                        "launch_calls": stats(launch),
                        "host_us_per_batch": round((sum(push) + sum(launch)) / (nd / per), 1)})
            if host_times is not None and name == "hash":
                host_times(buf)
                res[-1]["flush_parts_us_per_batch"] = {k: round(buf[i] / max(buf[5], 1.0), 1)
                                                       for i, k in enumerate(HOST_PARTS) if i != 5}
        out[name if grain is None else f"{name}_grain{grain}"] = res
        v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
