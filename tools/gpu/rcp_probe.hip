// rcp_probe.hip -- accuracy of v_rcp_f64 (__builtin_amdgcn_rcp on double) and of one / two
// Newton steps, over random z in [1e-3, 1e3] (the range of camera depths).  DESIGN.md §7.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstring>
__global__ void k(const double* z, double* e0, double* e1, double* e2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = z[i];
    double y = __builtin_amdgcn_rcp(x);
    double r = 1.0 / x;
    e0[i] = fabs(y - r) / r;
    double e = fma(-x, y, 1.0); double y1 = fma(y, e, y);
    e1[i] = fabs(y1 - r) / r;
    e = fma(-x, y1, 1.0); double y2 = fma(y1, e, y1);
    e2[i] = fabs(y2 - r) / r;
}
// Mantissa sweep: v_rcp_f64's relative error depends on the significand only, so z = 1 + i*2^-28
// over [1, 2) (plus the same sweep scaled by 2^-10 and 2^10) bounds it for every normal z the
// kernels see.  Max relative error as ordered bits (non-negative doubles order as integers).
__global__ void sweep(unsigned long long* mx, double scale) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double m = 0.0;
    for (int j = 0; j < 256; ++j) {  // 256 points per thread, one atomic each
        const double x = (1.0 + (double)(t * 256 + j) * 0x1p-28) * scale;
        const double y = __builtin_amdgcn_rcp(x);
        const double r = 1.0 / x;
        m = fmax(m, fabs(y - r) / r);
    }
    atomicMax(mx, (unsigned long long)__double_as_longlong(m));
}
int main() {
    {
        unsigned long long* dm;
        (void)hipMalloc(&dm, 8);
        const double scales[3] = {1.0, 0x1p-10, 0x1p10};
        for (double sc : scales) {
            (void)hipMemset(dm, 0, 8);
            sweep<<<(1 << 28) / (256 * 256), 256>>>(dm, sc);
            unsigned long long hm = 0;
            (void)hipMemcpy(&hm, dm, 8, hipMemcpyDeviceToHost);
            double e; memcpy(&e, &hm, 8);
            printf("rcp_f64 mantissa sweep (2^28 points, scale %g): max rel err %.3e (2^%.2f)\n", sc, e, log2(e));
        }
    }
    const int n = 1 << 22;
    double* h = (double*)malloc(n * 8);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = 1e-3 * pow(1e6, (double)(s >> 11) / 9007199254740992.0); }
    double *dz, *d0, *d1, *d2;
    hipMalloc(&dz, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
    hipMemcpy(dz, h, n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dz, d0, d1, d2, n);
    double* o = (double*)malloc(n * 8);
    double* outs[3] = {d0, d1, d2};
    for (int j = 0; j < 3; ++j) {
        hipMemcpy(o, outs[j], n * 8, hipMemcpyDeviceToHost);
        double mx = 0; for (int i = 0; i < n; ++i) mx = o[i] > mx ? o[i] : mx;
        printf("rcp_f64 + %d Newton steps: max rel err %.3e (2^%.1f)\n", j, mx, mx > 0 ? log2(mx) : -1e9);
    }
    return 0;
}
