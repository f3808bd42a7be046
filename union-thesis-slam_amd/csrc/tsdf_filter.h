// tsdf_filter.h -- host side of the certified f32 filter of the integrate kernels (the device
// side is project_part in tsdf_device.h; the derivation of the bound is there).  Plain C++ (no HIP),
// so that tools/check_f32_filter.cpp checks these very constants against the exact f64 path.
#pragma once
#include <cmath>

namespace tsdf {

// Per-frame constants of the filter (in Frame::ff).
struct F32Filter {
    float Tz32, Tx32, Ty32;   // RN32(T[10]), RN32(Tf[2]), RN32(Tf[6])
    float cxh, cyh;           // RN32(cx + 0.5), RN32(cy + 0.5)
    float hm32;               // a pixel index floor(s) is certain iff |fract(s) - 0.5| < hm32 (0.5 - margin)
    float zmin4, zmin8;       // ... and z32 >= zmin (z-parts of 4 / 8 steps): z > 0 certainly
    float zrej32;             // z32 < zrej32: z <= 0 certainly
    float t_rej, t_free;      // diff32 = d32 - z32 < t_rej: depth - z < -trunc certainly (no update);
                              // diff32 >= t_free: depth - z >= trunc certainly (dist = 1 exactly)
};

// |X - f x| of the folded f64 rows (Tf = RN(T * f), X = fma(Tf2, pz, fma(Tf1, py, fma(Tf0, px,
// Tf3)))): four roundings, each within 2^-53 of its operands' magnitudes, for world coordinates
// bounded by wmax (a factor 2 of slack).  Host.
inline double fold_error(const double* T, double fx, double fy, const double wmax[3]) {
    double e = 0.0;
    for (int r = 0; r < 2; ++r) {
        const double* t = T + 4 * r;
        const double s = fabs(t[0]) * wmax[0] + fabs(t[1]) * wmax[1] + fabs(t[2]) * wmax[2] + fabs(t[3]);
        e = fmax(e, 8.0 * 0x1p-53 * (r == 0 ? fx : fy) * s);
    }
    return e;
}

// f32 rounded towards -inf / +inf (host): thresholds that keep every f32 test conservative
inline float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}
inline float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// The filter's per-frame constants (host).  T: rows of world_to_cam; lo / hi: the volume's
// world box (voxel centres); vs, trunc: the volume's; wmax: bounds of |world coordinates|.
inline void f32_filter_consts(F32Filter* ff, const double* T, const double Tf[8], double fx, double fy, double cx,
                              double cy, int W, int H, const double lo[3], const double hi[3],
                              const double wmax[3], double vs, double trunc) {
    ff->Tz32 = (float)T[10];
    ff->Tx32 = (float)Tf[2];
    ff->Ty32 = (float)Tf[6];
    ff->cxh = (float)(cx + 0.5);
    ff->cyh = (float)(cy + 0.5);
    const double k24 = 0x1p-24, dz4 = 3.0 * vs, dz8 = 7.0 * vs, tz = fabs(T[10]);
    double rest = 0.0, dterm = 0.0;  // the margin's terms at the worse axis; dterm * dz / zmin
    for (int a = 0; a < 2; ++a) {
        const double c = a == 0 ? cx : cy, n = a == 0 ? W : H, tx = fabs(a == 0 ? Tf[2] : Tf[6]);
        const double q = fmax(fabs(c), fabs(n - c)) + 1.5;
        rest = fmax(rest, 7.0 * q + 1.5 * (fabs(c) + 0.5));
        dterm = fmax(dterm, 2.0 * (tx + q * tz));
    }
    // zmin: the dz term at half the rest (4-step parts; 8-step parts in proportion)
    const double zmin4 = fmax(dterm * dz4 / (0.5 * rest), 1e-3), zmin8 = zmin4 * dz8 / dz4;
    const double fold = fold_error(T, fx, fy, wmax);
    const double margin = 1.1 * (1.01 * k24 * 1.5 * rest + fold / zmin4 + 1e-9);
    ff->hm32 = margin < 0.5 ? f32_down(0.5 - margin) : 0.0f;  // (0: every step takes the f64 path)
    ff->zmin4 = f32_up(zmin4);
    ff->zmin8 = f32_up(zmin8);
    double zmax = 0.0;  // max |camera z| over the box: z is linear, so at a corner
    for (int c = 0; c < 8; ++c) {
        const double p[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        zmax = fmax(zmax, fabs(T[8] * p[0] + T[9] * p[1] + T[10] * p[2] + T[11]));
    }
    zmax = zmax * (1.0 + 1e-12) + vs;
    const double dmax = 65.535;  // u16 millimetres (f64 depth does not use the diff thresholds)
    const double eps = 1.1 * k24 * (2.8 * dmax + 3.0 * zmax + 2.0 * tz * dz8) + 1e-9;
    ff->zrej32 = f32_down(-1.1 * k24 * (2.0 * zmax + 2.0 * tz * dz8) - 1e-12);
    ff->t_rej = f32_down(-trunc - eps);
    ff->t_free = f32_up(trunc + eps);
}

}  // namespace tsdf
