"""tsdf_amd -- MI355X-native TSDF fusion hot path of DiWu9/Union-Thesis-SLAM.

Drop-in classes (put `union-thesis-slam_amd/` on sys.path, as the reference expects its repo
root on sys.path):

    from tsdf_amd.grid_fusion import TSDFVolume     # grid_fusion.TSDFVolume
    from tsdf_amd.hash_fusion import HashTable      # hash_fusion.HashTable

Both run on hand-written gfx950 HIP kernels through the C-ABI in include/tsdf_hip.h
(lib/libtsdf_hip.so, bound with ctypes in _ffi.py).  There is no CPU fallback.
"""
from . import _ffi  # noqa: F401

__all__ = ["grid_fusion", "hash_fusion", "data_structures", "scene"]
