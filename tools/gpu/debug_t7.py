"""Standalone replay of test_empty_and_invalid_depth_is_a_no_op with stats after each call."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "union-thesis-slam_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..", "tests")]
import numpy as np
from conftest import load_lounge, lounge_intrinsics
from tsdf_amd import grid_fusion as gf
C1 = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]
K = lounge_intrinsics()
vol = gf.TSDFVolume(np.array(C1), 0.04)
_, depth, rgb, pose = load_lounge(0)
vol.integrate(rgb, np.zeros_like(depth), K, pose)
print("call1", vol.stats(), flush=True)
away = pose.copy(); away[:3, 2] *= -1; away[:3, 0] *= -1
vol.integrate(rgb, depth, K, away)
print("call2", vol.stats(), flush=True)
T, W, C = vol.get_state()
print("ok", W.sum(), flush=True)
