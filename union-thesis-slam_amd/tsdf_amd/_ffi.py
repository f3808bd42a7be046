"""ctypes binding of libtsdf_hip.so (include/tsdf_hip.h).

This is the only way the package reaches the device: there is no CPU fallback.  If the HIP
library has not been built (`make -C union-thesis-slam_amd`, or __graft_entry__.build()) or no
gfx950 device is visible, the calls raise -- loudly, by design.

The reference binds its device code the same way, from Python at run time (PyCUDA
SourceModule + get_function, grid_fusion.py:69-144).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSDF_HIP_LIB") or os.path.join(_HERE, "lib", "libtsdf_hip.so")  # override: A/B builds of the same library

DEPTH_U16_MM, DEPTH_F64_M = 0, 1
COLOR_RGB8, COLOR_F32 = 0, 1
DEVICE_PTRS, ASYNC, DEPTH_INVALID_65535, DEFER = 1, 2, 4, 8

E_ARG, E_HIP, E_NODEV, E_CAPACITY, E_OOM = -1, -2, -3, -4, -5


class TSDFError(RuntimeError):
    """A C-ABI call returned an error code; the message is tsdf_last_error()."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[tsdf {code}] {msg}")
        self.code = code


class HIPLibraryMissing(ImportError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_int64), ("voxel_updates", ctypes.c_int64),
                ("bricks_visited", ctypes.c_int64), ("bricks_touched", ctypes.c_int64),
                ("blocks_allocated", ctypes.c_int64), ("probe_steps", ctypes.c_int64),
                ("probe_max", ctypes.c_int64), ("lookups", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("kernel_launches", ctypes.c_int64),
                ("bricks_skipped", ctypes.c_int64), ("list_errors", ctypes.c_int64),
                ("batch_voxels", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HashInfo(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_int64), ("used", ctypes.c_int64),
                ("tombstones", ctypes.c_int64), ("displaced", ctypes.c_int64),
                ("max_probe", ctypes.c_int64), ("blocks_in_pool", ctypes.c_int64),
                ("pool_capacity", ctypes.c_int64), ("entries", ctypes.c_int64), ("slots", ctypes.c_int64),
                ("pool_mapped", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_D = ctypes.c_double

# name -> argtypes (all return int)
SIGNATURES = {
    "tsdf_device_count": [_P],
    "tsdf_dense_create": [_P, _P, _P, _D, _D, _I, _P],
    "tsdf_dense_create_shard": [_P, _I, _I, _P, _D, _D, _I, _P],
    "tsdf_dense_extract_mesh": [_P, _P, _P],
    "tsdf_dense_get_mesh": [_P, _P, _P, _P, _P],
    "tsdf_dense_mesh_halo_rows": [_P, _I64, _P, _P],
    "tsdf_dense_extract_mesh_halo": [_P, _I64, _P, _I64, _P, _P, _I, _P, _P],
    "tsdf_dense_get_mesh_keys": [_P, _P],
    "tsdf_dense_get_rows": [_P, _P, _I64, _P, _P, _P, _I],
    "tsdf_mc_table": [_P, _P],
    "tsdf_frustum_bounds": [_P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P, _P],
    "tsdf_dense_destroy": [_P],
    "tsdf_dense_reset": [_P],
    "tsdf_dense_integrate": [_P, _P, _I, _P, _I, _I, _I, _P, _P, _D, _I],
    "tsdf_dense_integrate_batch": [_P, _I, _P, _I, _P, _I, _I, _I, _P, _P, _P, _I],
    "tsdf_dense_get": [_P, _P, _P, _P],
    "tsdf_dense_set": [_P, _P, _P, _P],
    "tsdf_dense_sync": [_P],
    "tsdf_dense_frames_per_launch": [_P, _P],
    "tsdf_dense_stats": [_P, _P, _I],
    "tsdf_dense_set_profiling": [_P, _I],
    "tsdf_hash_create": [_P, _P, _D, _D, _I64, _I64, _I, _I, _I, _I, _P],
    "tsdf_hash_destroy": [_P],
    "tsdf_hash_reset": [_P],
    "tsdf_hash_integrate": [_P, _P, _I, _P, _I, _I, _I, _P, _P, _I],
    "tsdf_hash_integrate_batch": [_P, _I, _P, _I, _P, _I, _I, _I, _P, _P, _I],
    "tsdf_hash_lookup": [_P, _P, _I64, _P, _P, _P, _P],
    "tsdf_hash_insert": [_P, _P, _I64, _P, _P, _P, _P, _P],
    "tsdf_hash_remove": [_P, _P, _I64, _P],
    "tsdf_hash_resize": [_P, _I64],
    "tsdf_hash_info": [_P, _P],
    "tsdf_hash_frames_per_launch": [_P, _P],
    "tsdf_hash_get_dense": [_P, _P, _P, _P],
    "tsdf_hash_to_dense": [_P, _P],
    "tsdf_hash_trim": [_P],
    "tsdf_hash_export_blocks": [_P, _P, _P, _P, _P, _P, _P, _I],
    "tsdf_hash_import_blocks": [_P, _P, _I64, _P, _P, _P, _P, _I],
    "tsdf_hash_sync": [_P],
    "tsdf_hash_stats": [_P, _P, _I],
    "tsdf_hash_set_profiling": [_P, _I],
    "tsdf_hash_keys": [_P, _I64, _I64, _I, _P, _I],
}

_lib = None


def load(path: str = LIB_PATH):
    """Load and type the library (no device call is made)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        # torch (when installed) brings its own libamdhip64.so.7; importing it FIRST makes the
        # dynamic linker bind this library to that same runtime (matching SONAME), so the
        # process has one HIP runtime and torch tensors / streams / synchronize() interoperate.
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(path):
        raise HIPLibraryMissing(
            f"{path} is missing: build it with `make -C union-thesis-slam_amd` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, args in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:  # an older build under A/B (TSDF_HIP_LIB): calling it fails loudly
            continue
        fn.argtypes = args
        fn.restype = ctypes.c_int
    for name in ("tsdf_last_error", "tsdf_build_id"):
        fn = getattr(lib, name)
        fn.argtypes = []
        fn.restype = ctypes.c_char_p
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise TSDFError(rc, lib.tsdf_last_error().decode(errors="replace"))


def ptr(a) -> ctypes.c_void_p | None:
    """Address of a C-contiguous ndarray (or None).  The returned pointer object holds a
    reference to the array (ndarray.ctypes.data_as), so a temporary passed straight into a call,
    e.g. ptr(f64(K, 9)), stays alive until the call returns."""
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(ctypes.c_void_p)


def build_id() -> str:
    """The loaded library's build id (sha256 prefix of its sources, tsdf_build_id)."""
    return load().tsdf_build_id().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    call("tsdf_device_count", ctypes.byref(n))
    return n.value


def f64(a, n):
    out = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    if out.size != n:
        raise ValueError(f"expected {n} values, got {out.size}")
    return out
