"""The deferred drop-in's host-side depth staging (csrc/tsdf_common.hip depth_mm_any, exported for
tests as tsdf_diag_depth_to_mm): f64 metres go to the device as u16 millimetres only when every
value is exactly RN(k / 1000) for an integer k in [0, 65535] -- the demos' `png / 1000.` -- so the
kernels' u16 conversion (fma(k, 0.001, k * C_LO), exact for every u16) reproduces the caller's
metres bit for bit; anything else stays f64.  Host code only: no GPU needed."""
import ctypes

import numpy as np
import pytest


def _conv(d):
    from tsdf_amd import _ffi
    lib = _ffi.load()
    f = lib.tsdf_diag_depth_to_mm
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    d = np.ascontiguousarray(d, np.float64)
    out = np.full(d.shape, 0xBEEF, np.uint16)
    rc = f(d.ctypes.data, d.size, out.ctypes.data)
    assert rc in (0, 1)
    return rc == 1, out


def test_every_millimetre_value_converts_exactly():
    k = np.arange(65536, dtype=np.uint16)
    ok, out = _conv(k.astype(np.float64) / 1000.0)  # 65536 values: the pooled path (>= 32K)
    assert ok and np.array_equal(out, k)
    ok, out = _conv(k[:1000].astype(np.float64) / 1000.0)  # the calling thread alone
    assert ok and np.array_equal(out, k[:1000])


@pytest.mark.parametrize("bad", [np.nan, -0.001, 65.536, np.inf, -np.inf, 1.0 + 2.0 ** -40])
def test_values_that_are_not_millimetres_refuse(bad):
    rng = np.random.default_rng(1)
    for n in (100, 640 * 480):
        d = rng.integers(0, 65536, n).astype(np.float64) / 1000.0
        d[rng.integers(0, n)] = bad
        assert not _conv(d)[0]


def test_one_ulp_off_refuses_and_negative_zero_passes():
    k = np.arange(1, 65536, dtype=np.float64)
    d = k / 1000.0
    for direction in (np.inf, -np.inf):
        e = d.copy()
        e[12345] = np.nextafter(e[12345], direction)
        assert not _conv(e)[0]
    z = np.zeros(50000)
    z[7] = -0.0  # depth > 0 and depth - z treat -0.0 and 0.0 alike
    ok, out = _conv(z)
    assert ok and not out.any()


def test_concurrent_callers_keep_their_own_verdicts():
    """Round-5 advisor finding: the copy pool is one per process and several threads may drive
    handles at once (ctypes releases the GIL).  A job's 'not exact millimetres' flag belongs to that
    job: exact and inexact frames converted from four threads at once each get their own answer."""
    import threading
    rng = np.random.default_rng(7)
    good = rng.integers(0, 65536, 640 * 480).astype(np.float64) / 1000.0
    bad = good.copy()
    bad[123456] += 1e-7
    errors = []

    def worker(t):
        for i in range(60):
            use_bad = (i + t) % 3 == 0
            ok, out = _conv(bad if use_bad else good)
            if ok == use_bad or (ok and not np.array_equal(out, np.round(good * 1000.0).astype(np.uint16))):
                errors.append((t, i, ok))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors
