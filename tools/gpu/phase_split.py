"""The integrate launch's phases as separate kernels, for a per-kernel time split under
`rocprofv3 --kernel-trace --stats` (call.sh `kt:phase_split.py`): the bench frames through the
in-line path (TSDF_PIPELINE=0: k_prep, k_cull, k_integrate, and for the hash k_free_unused, one
kernel each), dense and hash, 5 warm-up and 20 timed batches of the driver's window.  The fused
launch runs the same work overlapped; this only prices the parts.

    python tools/gpu/phase_split.py [texel: ignored by the in-line path]
"""
import json
import os
import sys
import time

os.environ["TSDF_PIPELINE"] = "0"
import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene  # noqa: E402


def main():
    F = 800
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
    ds, cs = 480 * 640 * 2, 480 * 640 * 3
    bnds = np.array([[0.0, 10.24]] * 3)
    out = {"build_id": _ffi.build_id()}
    for name, make in (("dense", lambda: grid_fusion.TSDFVolume(bnds.copy(), 0.02)),
                       ("hash", lambda: hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=1 << 15))):
        v = make()
        B = v.frames_per_launch()
        for s in range(0, 25 * B, B):  # 5 untimed + 20 timed batches (the profile takes them all)
            v.integrate_batch(depth.data_ptr() + s * ds, rgb.data_ptr() + s * cs, K, Tinv[s:s + B],
                              hw=(480, 640), device_ptrs=True, sync=name == "hash")
        v.sync()
        t0 = time.perf_counter()
        v.sync()
        out[name] = {"frames": 25 * B, "wall_check_s": time.perf_counter() - t0}
        v.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
