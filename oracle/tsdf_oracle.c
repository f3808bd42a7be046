/*
 * tsdf_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's integrate()
 * arithmetic, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * CHECKER.  It is never linked into, loaded by, or called from the product path
 * (union-thesis-slam_amd/), which fails loudly when its HIP library is missing.
 *
 * Parity status: PINNED.  tests/test_oracle_golden.py checks this file bit-for-bit against
 * golden vectors produced by the reference itself (tools/gen_golden.py, imported with
 * numba-typing-faithful helpers in the build container) and against the author's recorded
 * voxel-update counts.
 *
 * What it restates (all citations are into DiWu9/Union-Thesis-SLAM):
 *   vox2world      grid_fusion.py:170-181   p = f32( f64(origin_f32) + vs_f64 * f64(f32(idx)) )
 *   rigid_transform grid_fusion.py:363-368  np.dot(inv(pose), [p;1]) as OpenBLAS dgemm does it:
 *                                            c = fma(T3, 1, fma(T2, z, fma(T1, y, T0*x)))
 *   cam2pix        grid_fusion.py:183-197   u = int(rint((x*fx)/z + cx)), fx = f64(f32(K[0,0]))
 *   masks          grid_fusion.py:273-290   0<=u<W, 0<=v<H, z>0, d>0, d-z >= -trunc
 *   integrate_tsdf grid_fusion.py:199-212,293-299   mixed f32/f64 running average
 *   colour blend   grid_fusion.py:302-314   all-f32 decode/blend/round-half-even/encode
 *   Voxel.integrate data_structures/voxel.py:19-49   the hash path's f64 running average
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; no fast-math, so every operation rounds
 * exactly once, in the order written).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    int64_t dims[3];
    int64_t off[3]; /* global index of local voxel (0,0,0): slab sharding */
    const int64_t* xmap; /* if set, global x of local x row (cyclic column sharding) */
    float origin[3];
    double vs, trunc;
    double fx, fy, cx, cy; /* f64(f32(K)) as cam2pix casts intr to float32 first */
    double T[16];          /* inv(cam_pose), row-major, computed by NumPy on the host */
    int H, W;
} proj_t;

/* Project voxel (ix,iy,iz).  Returns 1 and fills *pix,*z when the voxel lands on a valid
 * pixel with z > 0 (grid_fusion.py:273-277). */
static inline int project(const proj_t* p, int64_t ix, int64_t iy, int64_t iz, int64_t* pix,
                          double* zout) {
    const int64_t gx = p->xmap ? p->xmap[ix] : ix + p->off[0];
    const float px = (float)((double)p->origin[0] + p->vs * (double)(float)gx);
    const float py = (float)((double)p->origin[1] + p->vs * (double)(float)(iy + p->off[1]));
    const float pz = (float)((double)p->origin[2] + p->vs * (double)(float)(iz + p->off[2]));
    const double* T = p->T;
    double c[3];
    for (int r = 0; r < 3; ++r) {
        const double* t = T + 4 * r;
        c[r] = fma(t[3], 1.0, fma(t[2], (double)pz, fma(t[1], (double)py, t[0] * (double)px)));
    }
    const double z = c[2];
    const double u = rint((c[0] * p->fx) / z + p->cx);
    const double v = rint((c[1] * p->fy) / z + p->cy);
    *zout = z;
    if (!(u >= 0.0 && u < (double)p->W && v >= 0.0 && v < (double)p->H && z > 0.0)) return 0;
    *pix = (int64_t)v * p->W + (int64_t)u;
    return 1;
}

static void fill_proj(proj_t* p, const int64_t* dims, const float* origin, double vs,
                      double trunc, const double* K, const double* Tinv, int H, int W) {
    memcpy(p->dims, dims, sizeof(p->dims));
    memset(p->off, 0, sizeof(p->off));
    p->xmap = NULL;
    memcpy(p->origin, origin, sizeof(p->origin));
    p->vs = vs;
    p->trunc = trunc;
    p->fx = (double)(float)K[0];
    p->fy = (double)(float)K[4];
    p->cx = (double)(float)K[2];
    p->cy = (double)(float)K[5];
    memcpy(p->T, Tinv, sizeof(p->T));
    p->H = H;
    p->W = W;
}

/* Dense grid integrate (grid_fusion.py:214-314, CPU branch).  State is C-order (X,Y,Z) f32.
 * depth: H*W float64 metres.  colour: H*W float32 folded B*65536+G*256+R (grid_fusion.py:232).
 * Returns the number of voxels updated; if `upd` is non-NULL, upd[i] = 1 for updated voxels. */
int64_t oracle_dense_integrate_rows(const int64_t* dims, const int64_t* off, const int64_t* xmap,
                                    const float* origin, double vs, double trunc, float* tsdf,
                                    float* weight, float* color, const double* depth,
                                    const float* color_im, int H, int W, const double* K,
                                    const double* Tinv, double ow, uint8_t* upd) {
    proj_t p;
    fill_proj(&p, dims, origin, vs, trunc, K, Tinv, H, W);
    if (off) memcpy(p.off, off, sizeof(p.off));
    p.xmap = xmap;
    const float ow32 = (float)ow; /* NumPy weak-scalar: Python float * f32 array stays f32 */
    int64_t n = 0;
    /* voxels are independent: (x, y) columns in parallel (OpenMP; the same result on any thread count) */
#pragma omp parallel for collapse(2) reduction(+ : n) schedule(static)
    for (int64_t ix = 0; ix < dims[0]; ++ix)
        for (int64_t iy = 0; iy < dims[1]; ++iy)
            for (int64_t iz = 0; iz < dims[2]; ++iz) {
                const int64_t i = (ix * dims[1] + iy) * dims[2] + iz;
                int64_t pix;
                double z;
                if (upd) upd[i] = 0;
                if (!project(&p, ix, iy, iz, &pix, &z)) continue;
                const double d = depth[pix];
                const double diff = d - z;
                if (!(d > 0.0 && diff >= -trunc)) continue;
                double dist = diff / trunc;
                if (dist > 1.0) dist = 1.0; /* np.minimum(1, .) */
                /* integrate_tsdf (grid_fusion.py:207-212) */
                const float w_old = weight[i];
                const float t_old = tsdf[i];
                const float w_new = (float)((double)w_old + ow);
                const float wt = w_old * t_old; /* f32 x f32 in numba */
                const float t_new = (float)(((double)wt + ow * dist) / (double)w_new);
                weight[i] = w_new;
                tsdf[i] = t_new;
                /* colour (grid_fusion.py:302-314), float32 throughout */
                const float oc = color[i];
                const float ob = floorf(oc / 65536.0f);
                const float og = floorf((oc - ob * 65536.0f) / 256.0f);
                const float orr = oc - ob * 65536.0f - og * 256.0f;
                const float nc = color_im[pix];
                const float nb = floorf(nc / 65536.0f);
                const float ng = floorf((nc - nb * 65536.0f) / 256.0f);
                const float nr = nc - nb * 65536.0f - ng * 256.0f;
                const float b = fminf(255.0f, rintf((w_old * ob + ow32 * nb) / w_new));
                const float g = fminf(255.0f, rintf((w_old * og + ow32 * ng) / w_new));
                const float r = fminf(255.0f, rintf((w_old * orr + ow32 * nr) / w_new));
                color[i] = b * 65536.0f + g * 256.0f + r;
                if (upd) upd[i] = 1;
                ++n;
            }
    return n;
}

int64_t oracle_dense_integrate_slab(const int64_t* dims, const int64_t* off, const float* origin,
                                    double vs, double trunc, float* tsdf, float* weight, float* color,
                                    const double* depth, const float* color_im, int H, int W,
                                    const double* K, const double* Tinv, double ow, uint8_t* upd) {
    return oracle_dense_integrate_rows(dims, off, NULL, origin, vs, trunc, tsdf, weight, color, depth,
                                       color_im, H, W, K, Tinv, ow, upd);
}

int64_t oracle_dense_integrate(const int64_t* dims, const float* origin, double vs, double trunc,
                               float* tsdf, float* weight, float* color, const double* depth,
                               const float* color_im, int H, int W, const double* K,
                               const double* Tinv, double ow, uint8_t* upd) {
    return oracle_dense_integrate_slab(dims, NULL, origin, vs, trunc, tsdf, weight, color, depth,
                                       color_im, H, W, K, Tinv, ow, upd);
}

/* Hash path integrate (hash_fusion.py:103-145 + voxel.py:19-49): same voxel set as the grid,
 * but each voxel is a Python Voxel holding float64 sdf/weight/colour and obs_weight is NOT
 * forwarded (hash_fusion.py:141,145: always 1).  State arrays are dense C-order f64 here (the
 * oracle does not need a sparse store); weight 0 means "no entry".
 * `new_key`, when non-NULL, receives 1 for voxels whose entry is created in this call, in the
 * reference's insertion order (C-order of valid voxels, hash_fusion.py:135). */
int64_t oracle_hash_integrate(const int64_t* dims, const float* origin, double vs, double trunc,
                              double* sdf, double* weight, double* color, const double* depth,
                              const float* color_im, int H, int W, const double* K,
                              const double* Tinv, uint8_t* upd, uint8_t* new_key) {
    proj_t p;
    fill_proj(&p, dims, origin, vs, trunc, K, Tinv, H, W);
    const double ow = 1.0;
    int64_t n = 0, i = 0;
    for (int64_t ix = 0; ix < dims[0]; ++ix)
        for (int64_t iy = 0; iy < dims[1]; ++iy)
            for (int64_t iz = 0; iz < dims[2]; ++iz, ++i) {
                int64_t pix;
                double z;
                if (upd) upd[i] = 0;
                if (new_key) new_key[i] = 0;
                if (!project(&p, ix, iy, iz, &pix, &z)) continue;
                const double d = depth[pix];
                const double diff = d - z;
                if (!(d > 0.0 && diff >= -trunc)) continue;
                double dist = diff / trunc;
                if (dist > 1.0) dist = 1.0;
                if (new_key && weight[i] == 0.0) new_key[i] = 1;
                const double w_old = weight[i];
                const double d_old = (w_old == 0.0) ? 1.0 : sdf[i];
                const double w_new = w_old + ow;
                sdf[i] = (d_old * w_old + dist * ow) / w_new;
                weight[i] = w_new;
                const double oc = color[i];
                const double ob = floor(oc / 65536.0);
                const double og = floor((oc - ob * 65536.0) / 256.0);
                const double orr = oc - ob * 65536.0 - og * 256.0;
                const float nc = color_im[pix];
                const float nb = floorf(nc / 65536.0f);
                const float ng = floorf((nc - nb * 65536.0f) / 256.0f);
                const float nr = nc - nb * 65536.0f - ng * 256.0f;
                /* obs_weight * new_b is Python float * np.float32 -> float32 (weak scalar) */
                const double b = fmin(255.0, rint((w_old * ob + (double)((float)ow * nb)) / w_new));
                const double g = fmin(255.0, rint((w_old * og + (double)((float)ow * ng)) / w_new));
                const double r = fmin(255.0, rint((w_old * orr + (double)((float)ow * nr)) / w_new));
                color[i] = b * 65536.0 + g * 256.0 + r;
                if (upd) upd[i] = 1;
                ++n;
            }
    return n;
}

/* hash_function (hash_fusion.py:182-190): ((x*P1) ^ (y*P2) ^ (z*P3)) floor-mod n.
 * int_bits = 64: NumPy int64 arithmetic (Linux, NumPy 2).  int_bits = 32: the wrapping int32
 * arithmetic of the author's Windows run. */
void oracle_hash_keys(const int64_t* xyz, int64_t n_pts, int64_t table_size, int int_bits,
                      int64_t* out) {
    const int64_t P1 = 73856093, P2 = 19349669, P3 = 83492791;
    for (int64_t k = 0; k < n_pts; ++k) {
        int64_t h;
        if (int_bits == 32) {
            const int32_t a = (int32_t)(uint32_t)((uint64_t)xyz[3 * k + 0] * (uint64_t)P1);
            const int32_t b = (int32_t)(uint32_t)((uint64_t)xyz[3 * k + 1] * (uint64_t)P2);
            const int32_t c = (int32_t)(uint32_t)((uint64_t)xyz[3 * k + 2] * (uint64_t)P3);
            h = (int64_t)(a ^ b ^ c);
        } else {
            h = (int64_t)(((uint64_t)xyz[3 * k + 0] * (uint64_t)P1) ^
                          ((uint64_t)xyz[3 * k + 1] * (uint64_t)P2) ^
                          ((uint64_t)xyz[3 * k + 2] * (uint64_t)P3));
        }
        int64_t m = h % table_size;
        if (m < 0) m += table_size; /* np.remainder: result has the divisor's sign */
        out[k] = m;
    }
}

/* get_view_frustum (grid_fusion.py:371-383) of one frame given its max depth, as a (3,5) array:
 * camera-frame points ((u - cx) * z / fx, (v - cy) * z / fy, z) for u in {0,0,0,W,W}, v in
 * {0,0,H,0,H}, z in {0,d,d,d,d} (NumPy elementwise order: subtract, multiply, divide), then
 * rigid_transform (363-368) = np.dot(cam_pose, [p;1]) as OpenBLAS dgemm (the FMA chain above). */
void oracle_view_frustum(double max_depth, int H, int W, const double* K, const double* pose,
                         double* out /* 3 x 5, row-major */) {
    const double us[5] = {0, 0, 0, (double)W, (double)W}, vs_[5] = {0, 0, (double)H, 0, (double)H};
    for (int j = 0; j < 5; ++j) {
        const double z = j == 0 ? 0.0 : max_depth;
        const double x = ((us[j] - K[2]) * z) / K[0];
        const double y = ((vs_[j] - K[5]) * z) / K[4];
        for (int r = 0; r < 3; ++r) {
            const double* t = pose + 4 * r;
            out[r * 5 + j] = fma(t[3], 1.0, fma(t[2], z, fma(t[1], y, t[0] * x)));
        }
    }
}
