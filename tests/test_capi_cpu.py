"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol that
include/tsdf_hip.h declares, and fails loudly (no CPU fallback) when no GPU is visible.
No compute call is made here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "tsdf_hip.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(tsdf_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from tsdf_amd import _ffi
    lib = _ffi.load()
    names = _declared()
    assert len(names) >= 27
    for n in names:
        assert hasattr(lib, n), n
    # every declared entry point is typed by the binding
    assert set(names) - {"tsdf_last_error", "tsdf_build_id"} == set(_ffi.SIGNATURES)


def test_build_id_names_the_sources():
    """tsdf_build_id() is the sha256 prefix of the sources the library was built from (the
    Makefile's BUILD_ID), so profiles can be matched to the library they measured."""
    import subprocess
    from tsdf_amd import _ffi
    bid = _ffi.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0
    pkg = os.path.join(REPO, "union-thesis-slam_amd")
    want = subprocess.run(["make", "-s", "-C", pkg, "--eval", "print-id: ; @echo $(BUILD_ID)", "print-id"],
                          capture_output=True, text=True, check=True).stdout.strip()
    assert bid == want, "the built library is stale: rebuild with make -C union-thesis-slam_amd"


def test_library_is_gfx950_code_object():
    path = os.path.join(REPO, "union-thesis-slam_amd", "tsdf_amd", "lib", "libtsdf_hip.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob
    assert b"k_integrate" in blob


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from tsdf_amd import _ffi, grid_fusion
    assert _ffi.device_count() == 0
    with pytest.raises(_ffi.TSDFError) as ei:
        grid_fusion.TSDFVolume(np.array([[0, 1.0], [0, 1.0], [0, 1.0]]), 0.1)
    assert ei.value.code == _ffi.E_NODEV


def test_argument_errors_are_reported_with_messages():
    from tsdf_amd import _ffi
    lib = _ffi.load()
    h = ctypes.c_void_p()
    dims = np.array([0, 4, 4], np.int64)
    rc = lib.tsdf_dense_create(_ffi.ptr(dims), None, _ffi.ptr(np.zeros(3, np.float32)), 0.1, 0.5, 0,
                               ctypes.byref(h))
    assert rc in (_ffi.E_ARG, _ffi.E_NODEV)
    assert lib.tsdf_last_error()
    rc = lib.tsdf_hash_keys(None, 3, 10, 64, None, 0)
    assert rc == _ffi.E_ARG and b"bad arguments" in lib.tsdf_last_error()


def test_host_encoding_duties():
    """Wrapper duties: uint16 depth goes as millimetres, float depth as float64
    metres untouched (the kernels read it as is); uint8 colour goes as is, other colour is folded
    exactly like grid_fusion.py:228-232."""
    from tsdf_amd import _ffi
    from tsdf_amd.grid_fusion import encode_color, encode_depth, volume_geometry
    mm = np.array([[0, 1, 999, 65535]], np.uint16)
    d = mm.astype(float) / 1000.0
    k, a = encode_depth(mm)
    assert k == _ffi.DEPTH_U16_MM and np.array_equal(a, mm)
    k, a = encode_depth(d)
    assert k == _ffi.DEPTH_F64_M and a is d  # no host pass, no copy
    k, a = encode_depth(d.astype(np.float32))
    assert k == _ffi.DEPTH_F64_M and a.dtype == np.float64
    rgb = np.arange(24, dtype=np.uint8).reshape(2, 4, 3)
    k, a = encode_color(rgb)
    assert k == _ffi.COLOR_RGB8 and a is not None
    k, a = encode_color(rgb.astype(np.float64) + 0.5)
    c = (rgb.astype(np.float32) + np.float32(0.5))
    assert k == _ffi.COLOR_F32 and np.array_equal(a, np.floor(c[..., 2] * 65536 + c[..., 1] * 256 + c[..., 0]))
    b = np.array([[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]])
    _, dims, origin, vs = volume_geometry(b, 0.04)
    assert list(dims) == [128, 128, 128] and origin.dtype == np.float32


def test_frame_stack_kinds_follow_dtypes():
    """integrate_batch never reinterprets host memory: kinds come from the dtypes and an
    explicit kind that disagrees is an error (no GPU needed)."""
    import numpy as np
    from tsdf_amd import _ffi
    from tsdf_amd.grid_fusion import frame_stack
    d16 = np.zeros((2, 4, 5), np.uint16)
    d64 = np.zeros((2, 4, 5), np.float64)
    rgb = np.zeros((2, 4, 5, 3), np.uint8)
    fold = np.zeros((2, 4, 5), np.float32)
    assert frame_stack(d16, None, rgb, None, False)[1::2] == (_ffi.DEPTH_U16_MM, _ffi.COLOR_RGB8)
    assert frame_stack(d64, None, fold, None, False)[1::2] == (_ffi.DEPTH_F64_M, _ffi.COLOR_F32)
    with pytest.raises(ValueError):
        frame_stack(d64, _ffi.DEPTH_U16_MM, rgb, None, False)
    with pytest.raises(ValueError):
        frame_stack(d64.astype(np.float32), None, rgb, None, False)
    with pytest.raises(ValueError):
        frame_stack(d16, None, rgb[:1], None, False)
    assert frame_stack(123, None, 456, None, True) == (123, _ffi.DEPTH_U16_MM, 456, _ffi.COLOR_RGB8)
