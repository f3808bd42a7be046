"""Host-side numerics the kernels rely on (CPU only)."""
import os
import subprocess

from conftest import REPO


def test_depth_mm_to_metres_conversion_is_exact_for_every_u16(tmp_path):
    """The kernels convert u16 millimetres with a two-term 1/1000, fma(m, C_HI, m*C_LO), instead
    of a division; it must equal NumPy's astype(float)/1000. for all 65536 inputs."""
    exe = os.path.join(tmp_path, "chk")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(REPO, "tools", "check_depth_conversion.c"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    assert "C_LO == RN(1/1000 - C_HI)" in out, out
    assert "two-term mismatches 0," in out, out
    assert "mul-only mismatches 0," not in out  # the plain product alone would NOT be exact


def test_frustum_planes_contain_the_valid_pixel_range():
    """The cull's half-spaces (tsdf_common.hip frustum_planes) restated: every point that
    projects to a valid pixel is inside all five planes."""
    import numpy as np
    rng = np.random.default_rng(0)
    fx = fy = 585.0
    cx, cy, W, H = 320.0, 240.0, 640, 480
    cam = [(0.0, 0.0, 1.0, 1e-4), (fx, 0.0, cx + 1.5, 0.0), (-fx, 0.0, W + 0.5 - cx, 0.0),
           (0.0, fy, cy + 1.5, 0.0), (0.0, -fy, H + 0.5 - cy, 0.0)]
    u = rng.uniform(-0.5, W - 0.5, 10000)
    v = rng.uniform(-0.5, H - 0.5, 10000)
    z = rng.uniform(1e-3, 20.0, 10000)
    x, y = (u - cx) * z / fx, (v - cy) * z / fy
    for a, b, c, e in cam:
        assert (a * x + b * y + c * z + e >= 0).all()


def test_markstein_quotient_matches_ieee_division(tmp_path):
    """tsdf_device.h div_rn (RN(1/b) + one FMA correction) must equal a / b on the operand
    ranges of the integrate kernels: diff / trunc and (w*t + dist) / (w + 1) for w < 65536."""
    exe = os.path.join(tmp_path, "cm")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(REPO, "tools", "check_markstein.c"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0 and "mismatches 0" in out.stdout, out.stdout


def test_f32_reciprocal_table_is_correctly_rounded():
    """The colour fast path takes RN32(1/n) as f32(RN64(1/n)) from the kernels' f64 table
    (n < kRcpBig = 65536); double rounding must not change any entry."""
    from fractions import Fraction
    import numpy as np
    for n in range(1, 65536):
        y32 = np.float32(np.float64(1.0) / np.float64(n))
        exact = Fraction(1, n)
        # y32 is RN32(1/n) iff no other float32 is closer (ties: even mantissa)
        lo, hi = np.nextafter(y32, np.float32(0)), np.nextafter(y32, np.float32(1))
        d = abs(Fraction(float(y32)) - exact)
        assert d <= abs(Fraction(float(lo)) - exact) and d <= abs(Fraction(float(hi)) - exact), n
        if d == abs(Fraction(float(lo)) - exact) or d == abs(Fraction(float(hi)) - exact):
            assert int(y32.view(np.uint32)) % 2 == 0, n

