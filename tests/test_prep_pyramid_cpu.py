"""The fused prep's max-depth pyramid (csrc/tsdf_device.h prep_vec_tile): levels 2-6 of a 64x64
tile are reduced by wave shuffles (ds_bpermute `__shfl_down`) with one workgroup barrier.  This
restates its lane arithmetic -- 512 threads, thread t = (r, c) = (t >> 4, t & 15) holding the two
level-1 texels (2c, r) and (2c + 1, r), shuffles within 64-lane waves, level 3 through LDS, wave 0
reducing levels 4-6 -- and checks every texel it writes against the plain 2x2 max pyramid the
cull's depth test assumes (a wrong lane offset would make the cull keep or drop the wrong bricks).
"""
import numpy as np


def shfl_down(v, delta):
    """__shfl_down within 64-lane waves: lane l reads lane l + delta, or its own value past the wave."""
    out = v.copy()
    n = len(v)
    for l in range(n):
        w0 = (l // 64) * 64
        src = l + delta
        if src < w0 + 64 and src < n:
            out[l] = v[src]
    return out


def emulate_tile(l1):
    """l1: the tile's 32x32 level-1 texels -> {level: {(x, y): value}} as the kernel writes them."""
    t = np.arange(512)
    r, c = t >> 4, t & 15
    ma = l1[r, 2 * c]
    mb = l1[r, 2 * c + 1]
    written = {L: {} for L in range(2, 7)}
    m2 = np.maximum(ma, mb)
    m2 = np.maximum(m2, shfl_down(m2, 16))
    for i in t[(r & 1) == 0]:
        written[2][(c[i], r[i] >> 1)] = m2[i]
    m3 = np.maximum(m2, shfl_down(m2, 1))
    m3 = np.maximum(m3, shfl_down(m3, 32))
    lds = np.zeros((8, 8), l1.dtype)
    for i in t[((r & 3) == 0) & ((c & 1) == 0)]:
        written[3][(c[i] >> 1, r[i] >> 2)] = m3[i]
        lds[r[i] >> 2, c[i] >> 1] = m3[i]
    lane = np.arange(64)
    lx, ly = lane & 7, lane >> 3
    m = lds[ly, lx].copy()
    m = np.maximum(m, shfl_down(m, 1))
    m = np.maximum(m, shfl_down(m, 8))
    for i in lane[((lx & 1) == 0) & ((ly & 1) == 0)]:
        written[4][(lx[i] >> 1, ly[i] >> 1)] = m[i]
    m = np.maximum(m, shfl_down(m, 2))
    m = np.maximum(m, shfl_down(m, 16))
    for i in lane[((lx & 3) == 0) & ((ly & 3) == 0)]:
        written[5][(lx[i] >> 2, ly[i] >> 2)] = m[i]
    m = np.maximum(m, shfl_down(m, 4))
    m = np.maximum(m, shfl_down(m, 32))
    written[6][(0, 0)] = m[0]
    return written


def test_shuffle_pyramid_equals_the_2x2_max_pyramid():
    rng = np.random.default_rng(5)
    for trial in range(20):
        l1 = rng.random((32, 32)).astype(np.float32)
        if trial % 3 == 0:  # invalid depth (0) over whole rows / columns, as past the image edge
            l1[rng.integers(0, 32):, :] = 0.0
            l1[:, rng.integers(0, 32):] = 0.0
        want = {1: l1}
        for L in range(2, 7):
            p = want[L - 1]
            want[L] = np.maximum(np.maximum(p[0::2, 0::2], p[0::2, 1::2]), np.maximum(p[1::2, 0::2], p[1::2, 1::2]))
        got = emulate_tile(l1)
        for L in range(2, 7):
            n = 32 >> (L - 1)
            assert len(got[L]) == n * n, L  # every texel of the level written once
            for (x, y), v in got[L].items():
                assert v == want[L][y, x], (L, x, y)
