"""How often the dense integrate's paths run on the bench workload (TSDF_DIAG build:
abtest/libdiag.so from tools/build_variant.sh diag -DTSDF_DIAG; TSDF_HIP_LIB selects it):
part-frames projected and with an update, steps whose pixel the bare-reciprocal fast path left
uncertain (redone with the reference's division) and the part-frames holding one, free-space skips
of the update's quotients, exact-path (non-canonical) part-frames.

    TSDF_HIP_LIB=abtest/libdiag.so PYTHONPATH=union-thesis-slam_amd python tools/gpu/diag_pairs.py [frames]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, scene  # noqa: E402

NAMES = ["part_frames", "part_frames_with_update", "uncertain_pixel_steps", "part_frames_with_uncertain",
         "free_space_skips", "exact_path_part_frames", "unused6", "unused7"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda", 0)
    poses = scene.trajectory(n, seed=0, radius_frac=scene.BENCH_RING)
    spheres = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((n, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, n, 50):
        d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    torch.cuda.synchronize()
    lib = _ffi.load()
    out = (ctypes.c_ulonglong * 8)()
    lib.tsdf_diag_counts(out)  # (clear)
    vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)
    vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), scene.intrinsics(), np.linalg.inv(poses),
                        hw=(480, 640), device_ptrs=True)
    lib.tsdf_diag_counts(out)
    st = vol.stats()
    res = {"frames": n, "build_id": _ffi.build_id(), "voxel_updates": st["voxel_updates"]}
    res.update({k: int(v) for k, v in zip(NAMES, out)})
    pf = max(res["part_frames"], 1)
    res["per_part_frame"] = {k: round(res[k] / pf, 4) for k in NAMES[1:]}
    res["voxel_efficiency"] = round(st["voxel_updates"] / (pf * 256), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
