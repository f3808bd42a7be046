"""Per-frame integrate() rate from host NumPy (the reference's call pattern), several passes, for
A/B of the host copy path (TSDF_COPY_THREADS):  python tools/gpu/dropin_rate.py [frames] [passes]
[TSDF_DEFER_MM values, e.g. 1,0: each measured in turn, twice, on fresh handles]"""
import contextlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene  # noqa: E402


def main():
    nd = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    poses = scene.trajectory(nd, seed=0, radius_frac=scene.BENCH_RING)
    d, c = scene.render(poses, scene.make_spheres(0, ring_frac=scene.BENCH_RING), seed=0,
                        device=torch.device("cuda", 0), depth_dtype=torch.int16)
    d64 = d.cpu().numpy().view(np.uint16).astype(np.float64) / 1000.0
    ch = c.cpu().numpy()
    K = scene.intrinsics()
    out = {"copy_threads": os.environ.get("TSDF_COPY_THREADS", "default"), "build_id": _ffi.build_id(),
           "copy_spin_us": os.environ.get("TSDF_COPY_SPIN_US", "default")}
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else [None]
    for rep in range(2 if modes[0] is not None else 1):
        for mode in modes:
            if mode is not None:
                os.environ["TSDF_DEFER_MM"] = mode  # (read when a handle is created)
            for name, mk in (("dense", lambda: grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)),
                             ("hash", lambda: hash_fusion.HashTable(np.array([[0.0, 10.24]] * 3), 0.02, 1 << 22,
                                                                    max_blocks=1 << 15))):
                with contextlib.redirect_stdout(sys.stderr):  # (the constructors' prints)
                    v = mk()
                v.integrate(ch[0], d64[0], K, poses[0])
                v.sync()
                rates = []
                for _ in range(passes):
                    t0 = time.perf_counter()
                    for i in range(nd):
                        v.integrate(ch[i], d64[i], K, poses[i])
                    v.sync()
                    rates.append(round(nd / (time.perf_counter() - t0), 1))
                key = name if mode is None else f"{name}_mm{mode}_rep{rep}"
                out[key] = rates
                v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
