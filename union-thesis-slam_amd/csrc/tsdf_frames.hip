// tsdf_frames.hip -- frame-level utilities around the integrate path:
// volume bounds from the union of the frames' view frustums, the MI355X replacement of the
// demo loop grid_demo1.py:50-64 / hash_demo1.py:93-107 over get_view_frustum
// (grid_fusion.py:371-383).
//
// Two kernels per chunk of frames: k_frame_max reduces each frame's depth to its maximum (an
// HBM-streaming reduction: 2 B/px for u16, 8 B/px for f64), k_frustum turns each maximum and
// pose into the 5 frustum points -- with the reference's f64 operation order and the OpenBLAS
// dgemm FMA chain of rigid_transform -- and folds them into 6 order-preserving keys with
// atomicMin/atomicMax.  Maxima and bounds are exact: identical to the reference's f64 values.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "tsdf_host.h"

using namespace tsdf;

namespace {

// Order-preserving map of doubles to u64 (a < b <=> key(a) < key(b) for non-NaN values).
__device__ __host__ inline unsigned long long dkey(double x) {
    unsigned long long b;
    memcpy(&b, &x, 8);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __host__ inline double dval(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
    double x;
    memcpy(&x, &b, 8);
    return x;
}

constexpr int kMaxWG = 256;

// Max depth of frame blockIdx.y (metres as the reference sees it: f64(mm) / 1000, or the f64
// value), as a key in keys[frame].  invalid_65535: the 7-Scenes convention of the demos
// (grid_demo1.py:82: 65.535 m -> 0).
template <int DK>
__global__ __launch_bounds__(kMaxWG) void k_frame_max(const void* depth, long long npx, int invalid_65535,
                                                      unsigned long long* keys) {
    const long long f = blockIdx.y;
    unsigned long long best = dkey(DK == 0 ? 0.0 : -1.0 / 0.0);
    if (DK == 0) {
        const unsigned short* d = (const unsigned short*)depth + f * npx;
        unsigned m = 0;
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < npx;
             i += (long long)gridDim.x * blockDim.x) {
            const unsigned v = d[i];
            m = (invalid_65535 && v == 65535u) ? m : max(m, v);
        }
        best = dkey((double)m / 1000.0);
    } else {
        const double* d = (const double*)depth + f * npx;
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < npx;
             i += (long long)gridDim.x * blockDim.x) {
            const double v = d[i];
            if (v == v) best = max(best, dkey(v));  // np.max would propagate a NaN; skip it
        }
    }
    for (int o = 32; o > 0; o >>= 1) best = max(best, (unsigned long long)__shfl_xor(best, o));
    __shared__ unsigned long long s[kMaxWG / 64];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = max(best, s[w]);
        atomicMax(keys + f, best);
    }
}

// One thread per frame: grid_fusion.py:371-383 then the demo's min/max (keys[0..2] = min x,y,z;
// keys[3..5] = max x,y,z).
__global__ void k_frustum(int n, int H, int W, const double* __restrict__ K,
                          const double* __restrict__ poses, const unsigned long long* __restrict__ maxk,
                          double* __restrict__ pts, unsigned long long* bkeys) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    const double dmax = dval(maxk[f]);
    const double* T = poses + 16 * (long long)f;
    const double us[5] = {0.0, 0.0, 0.0, (double)W, (double)W};
    const double vs[5] = {0.0, 0.0, (double)H, 0.0, (double)H};
    double lo[3] = {1.0 / 0.0, 1.0 / 0.0, 1.0 / 0.0}, hi[3] = {-1.0 / 0.0, -1.0 / 0.0, -1.0 / 0.0};
    for (int j = 0; j < 5; ++j) {
        const double z = j == 0 ? 0.0 : dmax;
        const double x = ((us[j] - K[2]) * z) / K[0];
        const double y = ((vs[j] - K[5]) * z) / K[4];
        for (int r = 0; r < 3; ++r) {
            const double* t = T + 4 * r;
            const double c = fma(t[3], 1.0, fma(t[2], z, fma(t[1], y, t[0] * x)));
            if (pts) pts[15 * (long long)f + 5 * r + j] = c;
            lo[r] = fmin(lo[r], c);
            hi[r] = fmax(hi[r], c);
        }
    }
    for (int r = 0; r < 3; ++r) {
        atomicMin(bkeys + r, dkey(lo[r]));
        atomicMax(bkeys + 3 + r, dkey(hi[r]));
    }
}

__global__ void k_init_keys(unsigned long long* k, int n, unsigned long long v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = v;
}

}  // namespace

extern "C" {

int tsdf_frustum_bounds(const void* depth, int depth_kind, int n_frames, int height, int width,
                        const double K[9], const double* cam_poses, int flags, int device,
                        double* max_depth, double* frustum_pts, double bounds[6]) {
    if (!depth || !K || !cam_poses || !bounds) return set_error(TSDF_E_ARG, "null pointer");
    if (depth_kind != TSDF_DEPTH_U16_MM && depth_kind != TSDF_DEPTH_F64_M)
        return set_error(TSDF_E_ARG, "bad depth_kind %d", depth_kind);
    if (n_frames < 0 || height <= 0 || width <= 0) return set_error(TSDF_E_ARG, "bad frame count/size");
    if (n_frames == 0) return TSDF_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return set_error(TSDF_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return set_error(TSDF_E_ARG, "device %d out of range [0,%d)", device, ndev);
    const int dev = device;
    TSDF_HIP(hipSetDevice(dev));
    const long long npx = (long long)height * width;
    const size_t esz = depth_kind == TSDF_DEPTH_U16_MM ? 2 : 8;
    const bool dptr = flags & TSDF_DEVICE_PTRS;
    const int inval = (flags & TSDF_DEPTH_INVALID_65535) ? 1 : 0;
    const int chunk = dptr ? n_frames : std::min(n_frames, 64);
    hipStream_t s = nullptr;
    unsigned long long *maxk = nullptr, *bk = nullptr;
    double *dK = nullptr, *dpose = nullptr, *dpts = nullptr;
    void* stage = nullptr;
    int cu = 256;
    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&maxk, sizeof(unsigned long long) * n_frames);
    if (e == hipSuccess) e = hipMalloc(&bk, sizeof(unsigned long long) * 6);
    if (e == hipSuccess) e = hipMalloc(&dK, sizeof(double) * 9);
    if (e == hipSuccess) e = hipMalloc(&dpose, sizeof(double) * 16 * n_frames);
    if (e == hipSuccess && frustum_pts) e = hipMalloc(&dpts, sizeof(double) * 15 * n_frames);
    if (e == hipSuccess && !dptr) e = hipMalloc(&stage, esz * npx * chunk);
    if (e == hipSuccess) e = hipMemcpyAsync(dK, K, sizeof(double) * 9, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dpose, cam_poses, sizeof(double) * 16 * n_frames, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_init_keys, dim3((n_frames + 255) / 256), dim3(256), 0, s, maxk, n_frames, 0ull);
        hipLaunchKernelGGL(k_init_keys, dim3(1), dim3(64), 0, s, bk, 3, ~0ull);
        hipLaunchKernelGGL(k_init_keys, dim3(1), dim3(64), 0, s, bk + 3, 3, 0ull);
        e = hipGetLastError();
    }
    // enough workgroups per frame to stream the image at full HBM rate
    const unsigned per_frame = (unsigned)std::max(1ll, std::min<long long>((npx + 4095) / 4096, std::max(1, 4 * cu / std::max(1, chunk))));
    for (int f0 = 0; f0 < n_frames && e == hipSuccess; f0 += chunk) {
        const int m = std::min(chunk, n_frames - f0);
        const char* src = (const char*)depth + esz * npx * f0;
        if (!dptr) {
            e = hipMemcpyAsync(stage, src, esz * npx * m, hipMemcpyHostToDevice, s);
            src = (const char*)stage;
        }
        if (e != hipSuccess) break;
        if (depth_kind == TSDF_DEPTH_U16_MM)
            hipLaunchKernelGGL(k_frame_max<0>, dim3(per_frame, m), dim3(kMaxWG), 0, s, (const void*)src, npx, inval, maxk + f0);
        else
            hipLaunchKernelGGL(k_frame_max<1>, dim3(per_frame, m), dim3(kMaxWG), 0, s, (const void*)src, npx, inval, maxk + f0);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_frustum, dim3((n_frames + 63) / 64), dim3(64), 0, s, n_frames, height, width,
                           (const double*)dK, (const double*)dpose, (const unsigned long long*)maxk, dpts, bk);
        e = hipGetLastError();
    }
    std::vector<unsigned long long> hk(n_frames), hb(6);
    if (e == hipSuccess) e = hipMemcpyAsync(hb.data(), bk, sizeof(unsigned long long) * 6, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && max_depth) e = hipMemcpyAsync(hk.data(), maxk, sizeof(unsigned long long) * n_frames, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && frustum_pts) e = hipMemcpyAsync(frustum_pts, dpts, sizeof(double) * 15 * n_frames, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    for (void* p : {(void*)maxk, (void*)bk, (void*)dK, (void*)dpose, (void*)dpts, stage})
        if (p) (void)hipFree(p);
    if (s) (void)hipStreamDestroy(s);
    TSDF_HIP(e);
    if (max_depth)
        for (int f = 0; f < n_frames; ++f) max_depth[f] = dval(hk[f]);
    // the demo's np.minimum / np.maximum with the incoming bounds (it starts from zeros)
    for (int r = 0; r < 3; ++r) {
        bounds[2 * r] = std::fmin(bounds[2 * r], dval(hb[r]));
        bounds[2 * r + 1] = std::fmax(bounds[2 * r + 1], dval(hb[3 + r]));
    }
    return TSDF_OK;
}

}  // extern "C"
