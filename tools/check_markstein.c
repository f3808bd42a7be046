/* Checks the kernels' division shortcut (tsdf_device.h div_rn): with y = RN(1/b),
 * q0 = RN(a*y), r = fma(-q0, b, a), q = fma(r, y, q0) equals the IEEE quotient a / b.
 *   (1) dist = diff / trunc for the truncation margins of every tested volume, diff over the
 *       integrate range [-trunc, 70 m] (random, plus values next to multiples of trunc);
 *   (2) tsdf = (w*t + dist) / (w + 1) for integer weights 1..65535 (the reciprocal table, LDS
 *       part < 4096 and HBM part), numerators over [-(w+2), w+2] (random, plus values next to
 *       multiples of the divisor).
 * Prints "markstein checked N mismatches M" (expected M = 0).  Build: gcc -O2 -ffp-contract=off -lm. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static double urand(void) { /* [0,1) */
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return (double)(s >> 11) * 0x1.0p-53;
}
static double div_rn(double a, double b, double y) {
    const double q0 = a * y;
    const double r = fma(-q0, b, a);
    return fma(r, y, q0);
}
static long check(double a, double b, double y) {
    /* subnormal numerators are outside the theorem (underflow) and cannot occur in the kernels:
     * diff = depth - z and w*t + dist are 0 or differences/sums of normal doubles >= 2^-80 */
    if (a != 0.0 && fabs(a) < 0x1.0p-1022) return 0;
    volatile double q = a / b;
    return div_rn(a, b, y) != q;
}

int main(void) {
    long bad = 0, n = 0;
    const double truncs[] = {5 * 0.02, 5 * 0.04, 5 * 0.08, 5 * 0.01, 5 * 0.03, 5 * 0.0123, 5 * 0.05, 0.1, 0.3};
    for (unsigned t = 0; t < sizeof(truncs) / sizeof(truncs[0]); ++t) {
        const double b = truncs[t], y = 1.0 / b;
        for (long i = 0; i < 2000000; ++i, ++n) bad += check(-b + (70.0 + b) * urand(), b, y);
        for (long k = -1; k < 700; ++k) {  /* near exact multiples: a = k*b +- few ulps */
            double a = (double)k * b;
            for (int j = 0; j < 8; ++j, ++n) {
                bad += check(a, b, y);
                a = nextafter(a, j < 4 ? INFINITY : -INFINITY);
            }
        }
    }
    for (int w = 1; w < 65536; ++w) {
        const double b = (double)w, y = 1.0 / b, span = b + 2.0;
        const int nr = w < 4096 ? 2000 : 150;
        for (int i = 0; i < nr; ++i, ++n) bad += check(-span + 2.0 * span * urand(), b, y);
        for (int k = -w - 1; k <= w + 1; k += 1 + w / 64) {
            double a = (double)k * b + 0.5 * b * (k & 1);
            for (int j = 0; j < 6; ++j, ++n) {
                bad += check(a, b, y);
                a = nextafter(a, j < 3 ? INFINITY : -INFINITY);
            }
        }
    }
    printf("markstein checked %ld mismatches %ld\n", n, bad);
    return bad != 0;
}
