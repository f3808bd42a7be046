"""Part-frame pairs the dense integrate computes vs those with a valid voxel (TSDF_DIAG build:
abtest/libdiag.so from tools/build_variant.sh diag -DTSDF_DIAG), on the bench workload."""
import json
import sys

import numpy as np
import torch

from tsdf_amd import grid_fusion, scene


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
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
    vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.02)
    vol.integrate_batch(depth.data_ptr(), rgb.data_ptr(), scene.intrinsics(), np.linalg.inv(poses),
                        hw=(480, 640), device_ptrs=True)
    st = vol.stats()
    st["pairs_computed"], st["pairs_valid"] = st.pop("probe_steps"), st.pop("lookups")
    st["valid_frac"] = st["pairs_valid"] / max(st["pairs_computed"], 1)
    st["voxel_steps_computed"] = st["pairs_computed"] * 256
    st["voxel_efficiency"] = st["voxel_updates"] / max(st["voxel_steps_computed"], 1)
    print(json.dumps(st))


if __name__ == "__main__":
    main()
