// check_f32_filter.cpp -- CPU check of the integrate kernels' certified f32 filter
// (csrc/tsdf_device.h project_part; constants from csrc/tsdf_filter.h, included as is).
//
// For random camera poses around / inside a volume and random voxels of it, the filter's f32
// arithmetic is replayed operation for operation (fmaf where the kernel packs v_pk_fma_f32,
// v_rcp_f32 modelled as RN(1/z) and as its neighbours one ulp either side, v_fract_f32,
// v_cvt_flr_i32_f32), and every decision it takes as certain is compared with the reference's f64
// path (grid_fusion.py:262-290 in the operation order of SURVEY §8(a)): the pixel index, z > 0,
// depth - z >= -trunc and depth - z >= trunc.  Also reported: the largest error of the f32 pixel
// coordinate relative to the margin, the share of uncertain steps and of steps in the band.
//   g++ -O2 -ffp-contract=off -I union-thesis-slam_amd/csrc tools/check_f32_filter.cpp -o chk && ./chk
// Exit status 1 on any wrong certain decision.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

#include "tsdf_filter.h"

using namespace tsdf;

struct Case {
    const char* name;
    double origin[3];
    double vs;
    int dims[3];
    int W, H;
    double fx, fy, cx, cy;
    bool inside;  // camera inside the volume (else around it)
};

static double vox_world(float origin, double vs, int g) { return (double)(float)((double)origin + vs * (double)g); }

static void random_pose(std::mt19937_64& rng, const double c[3], double T[16]) {
    // camera-to-world: random rotation (uniform quaternion), centre c; T = its inverse (rigid)
    std::normal_distribution<double> n(0.0, 1.0);
    double q[4] = {n(rng), n(rng), n(rng), n(rng)};
    const double l = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double& x : q) x /= l;
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                         2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                         2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
    for (int r = 0; r < 3; ++r) {  // inverse: R^T, -R^T c
        for (int k = 0; k < 3; ++k) T[4 * r + k] = R[3 * k + r];
        T[4 * r + 3] = -(R[0 * 3 + r] * c[0] + R[1 * 3 + r] * c[1] + R[2 * 3 + r] * c[2]);
    }
    T[12] = T[13] = T[14] = 0.0;
    T[15] = 1.0;
}

int main(int argc, char** argv) {
    const long long per_case = argc > 1 ? atoll(argv[1]) : 4000000;
    const Case cases[] = {
        {"bench 512^3 @ 2 cm, 640x480, inside", {0.0, 0.0, 0.0}, 0.02, {512, 512, 512}, 640, 480, 585, 585, 320, 240, true},
        {"lounge bounds @ 2 cm, around", {-4.22106438, -2.6663104, 0.0}, 0.02, {405, 264, 289}, 640, 480, 585, 585, 320, 240, false},
        {"10 km from the origin @ 2 cm, inside", {1e4, -7e3, 5e3}, 0.02, {512, 512, 512}, 640, 480, 585, 585, 320, 240, true},
        {"1024^3 @ 1 cm, odd centre", {0.0, 0.0, 0.0}, 0.01, {1024, 1024, 1024}, 640, 480, 571.3, 570.9, 319.37, 241.81, true},
        {"128^3 @ 4 cm, 1280x960", {-2.56, -2.56, 0.0}, 0.04, {128, 128, 128}, 1280, 960, 1170, 1170, 640, 480, false},
    };
    int bad = 0;
    for (const Case& cs : cases) {
        std::mt19937_64 rng(12345);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        const float origin[3] = {(float)cs.origin[0], (float)cs.origin[1], (float)cs.origin[2]};
        const double trunc = 5.0 * cs.vs;
        double lo[3], hi[3], wmax[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = (double)origin[a];
            hi[a] = (double)origin[a] + cs.vs * (cs.dims[a] - 1);
            wmax[a] = std::fmax(std::fabs(lo[a]), std::fabs(hi[a])) + cs.vs + 1.0;
        }
        const double fx = (double)(float)cs.fx, fy = (double)(float)cs.fy, cx = (double)(float)cs.cx,
                     cy = (double)(float)cs.cy;
        long long n = 0, in_img = 0, slow = 0, band = 0, wrong = 0, checked_rej = 0, checked_free = 0;
        double worst = 0.0, margin_used = 0.0;
        const int poses = 400;
        for (int pi = 0; pi < poses; ++pi) {
            double c[3];
            for (int a = 0; a < 3; ++a) {
                const double ext = hi[a] - lo[a];
                c[a] = cs.inside ? lo[a] + ext * (0.1 + 0.8 * U(rng)) : lo[a] + ext * (-0.3 + 1.6 * U(rng));
            }
            double T[16];
            random_pose(rng, c, T);
            double Tf[8];
            for (int j = 0; j < 4; ++j) {
                Tf[j] = T[j] * fx;
                Tf[4 + j] = T[4 + j] * fy;
            }
            F32Filter ff;
            f32_filter_consts(&ff, T, Tf, fx, fy, cx, cy, cs.W, cs.H, lo, hi, wmax, cs.vs, trunc);
            margin_used = 0.5 - (double)ff.hm32;
            for (long long t = 0; t < per_case / poses; ++t) {
                // a voxel part: column (gx, gy), first step gz0 (4-step parts), step k
                const int gx = (int)(U(rng) * cs.dims[0]), gy = (int)(U(rng) * cs.dims[1]);
                const int gz0 = 4 * (int)(U(rng) * (cs.dims[2] / 4)), k = (int)(U(rng) * 4);
                const double px = vox_world(origin[0], cs.vs, gx), py = vox_world(origin[1], cs.vs, gy);
                const double pz0 = vox_world(origin[2], cs.vs, gz0), pz = vox_world(origin[2], cs.vs, gz0 + k);
                // the reference (f64, OpenBLAS's dgemm chain, then (x*fx)/z + cx and rint)
                const double a0 = std::fma(T[1], py, T[0] * px), a1 = std::fma(T[5], py, T[4] * px);
                const double a2 = std::fma(T[9], py, T[8] * px);
                const double x = T[3] + std::fma(T[2], pz, a0), y = T[7] + std::fma(T[6], pz, a1);
                const double z = T[11] + std::fma(T[10], pz, a2);
                const double ux = (x * fx) / z + cx, uy = (y * fy) / z + cy;
                const long long eu = (long long)std::rint(ux), ev = (long long)std::rint(uy);
                // the filter (project_part)
                const float Z0 = (float)(T[11] + std::fma(T[10], pz0, a2));
                const float X0 = (float)std::fma(Tf[2], pz0, std::fma(Tf[1], py, std::fma(Tf[0], px, Tf[3])));
                const float Y0 = (float)std::fma(Tf[6], pz0, std::fma(Tf[5], py, std::fma(Tf[4], px, Tf[7])));
                const float dz = (float)(pz - pz0);
                const float zz = std::fmaf(dz, ff.Tz32, Z0), xx = std::fmaf(dz, ff.Tx32, X0),
                            yy = std::fmaf(dz, ff.Ty32, Y0);
                ++n;
                if (zz < ff.zrej32 && z > 0.0) {
                    ++wrong;
                    if (wrong < 10) printf("  z rejected wrongly: z %.9g z32 %.9g\n", z, zz);
                }
                const bool zok = zz >= ff.zmin4;
                if (zok && !(z > 0.0)) {
                    ++wrong;
                    if (wrong < 10) printf("  z accepted wrongly: z %.9g z32 %.9g\n", z, zz);
                }
                const bool near_img = eu >= -1 && eu <= cs.W && ev >= -1 && ev <= cs.H;
                if (zok && near_img) {
                    ++in_img;
                    const float r0 = 1.0f / zz;  // RN(1/z) and the neighbours v_rcp_f32 may return
                    const float rs[3] = {r0, std::nextafterf(r0, 0.0f), std::nextafterf(r0, INFINITY)};
                    bool fine_all = true, any_fine = false;
                    for (float rz : rs) {
                        const float sx = std::fmaf(xx, rz, ff.cxh), sy = std::fmaf(yy, rz, ff.cyh);
                        const float fu = (sx - std::floor(sx)) - 0.5f, fv = (sy - std::floor(sy)) - 0.5f;
                        const bool fine = std::fabs(fu) < ff.hm32 && std::fabs(fv) < ff.hm32;
                        fine_all &= fine;
                        any_fine |= fine;
                        worst = std::fmax(worst, std::fmax(std::fabs((double)sx - (ux + 0.5)),
                                                           std::fabs((double)sy - (uy + 0.5))) / margin_used);
                        if (fine && ((long long)std::floor(sx) != eu || (long long)std::floor(sy) != ev)) {
                            ++wrong;
                            if (wrong < 10) printf("  pixel wrong: (%lld,%lld) vs (%.9f, %.9f) z %.6g\n", eu, ev, sx, sy, z);
                        }
                    }
                    if (!fine_all) ++slow;
                    // depth: a random u16 around this voxel's z (the band and both limits often)
                    const double zt = z + trunc * (U(rng) * 4.0 - 2.0);
                    const unsigned raw = (unsigned)std::fmin(65535.0, std::fmax(1.0, std::rint(zt * 1000.0)));
                    const double d = (double)raw / 1000.0, diff = d - z;
                    const float d32 = (float)raw * 0.001f, df = d32 - zz;
                    if (df < ff.t_rej) {
                        ++checked_rej;
                        if (diff >= -trunc) ++wrong;
                    } else if (df >= ff.t_free) {
                        ++checked_free;
                        if (diff < trunc) ++wrong;
                    } else {
                        ++band;
                    }
                }
            }
        }
        printf("%-40s margin %.3g px  worst |s - exact| / margin %.3f  uncertain %.4f%%  band %.2f%%  "
               "(%lld steps, %lld near the image, %lld certain rejects, %lld certain free)  wrong %lld\n",
               cs.name, margin_used, worst, 100.0 * slow / std::fmax(1.0, (double)in_img),
               100.0 * band / std::fmax(1.0, (double)in_img), n, in_img, checked_rej, checked_free, wrong);
        if (wrong || worst >= 1.0) bad = 1;
    }
    printf(bad ? "FAILED\n" : "all certain decisions exact, wrong 0\n");
    return bad;
}
