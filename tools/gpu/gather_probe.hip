// gather_probe.hip -- cost of the integrate kernel's per-step image gathers on gfx950: 64 lanes of
// an 8x8 voxel column projected ~4 px apart onto a 640x480 image, gathered as u16 + u32 (depth and
// packed colour, two instructions) or as one u64 (both in one texel).  Every CU runs 16 waves;
// prints ns per wave-gather-step per CU (lower = better) for each form.
//   hipcc -O3 --offload-arch=gfx950 tools/gpu/gather_probe.hip -o tools/gpu/gather_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 640, H = 480, kSteps = 512;

__device__ inline unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// pixel of lane (lx, ly) at step s: a 4-px lattice rotated by a per-wave angle, jittered
__device__ inline int pix(int s, int lane, int seed, int spread) {
    const unsigned h = hash32((unsigned)(s * 7919 + seed));
    const int u0 = 40 + (int)(h % (W - 80)), v0 = 40 + (int)((h >> 12) % (H - 80));
    const int lx = lane >> 3, ly = lane & 7;
    const int du = (lx * spread + ly * (spread / 4)) % 36, dv = (ly * spread - lx * (spread / 4) + 36) % 36;
    return (v0 + dv - 18) * W + (u0 + du - 18);
}

template <int MODE>  // 0: u16 + u32 ; 1: u64 ; 2: u16 only ; 3: u32 only
__global__ __launch_bounds__(1024) void k(const unsigned short* d16, const unsigned* c32,
                                          const unsigned long long* dc64, unsigned* out, int spread) {
    const int lane = threadIdx.x & 63;
    const int seed = blockIdx.x * 16 + (threadIdx.x >> 6);
    unsigned acc = 0;
    for (int s = 0; s < kSteps; s += 4) {
        unsigned a[4], b[4];
        unsigned long long c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = pix(s + k, lane, seed, spread);
            if (MODE == 0) { a[k] = d16[p]; b[k] = c32[p]; }
            if (MODE == 1) c[k] = dc64[p];
            if (MODE == 2) a[k] = d16[p];
            if (MODE == 3) b[k] = c32[p];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (MODE == 0) acc += a[k] ^ b[k];
            if (MODE == 1) acc += (unsigned)c[k] ^ (unsigned)(c[k] >> 32);
            if (MODE == 2) acc += a[k];
            if (MODE == 3) acc += b[k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    unsigned short* d16; unsigned* c32; unsigned long long* dc64; unsigned* out;
    (void)hipMalloc(&d16, W * H * 2); (void)hipMalloc(&c32, W * H * 4); (void)hipMalloc(&dc64, W * H * 8);
    (void)hipMemset(d16, 1, W * H * 2); (void)hipMemset(c32, 1, W * H * 4); (void)hipMemset(dc64, 1, W * H * 8);
    const int blocks = 256 * 4;  // 4 workgroups of 1024 threads per CU: 64 waves -> enough to saturate
    (void)hipMalloc(&out, sizeof(unsigned) * blocks * 1024);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char* names[4] = {"u16 + u32", "u64", "u16 only", "u32 only"};
    for (int spread : {4, 8}) {
        for (int m = 0; m < 4; ++m) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(1024), 0, 0, d16, c32, dc64, out, spread);
                if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(1024), 0, 0, d16, c32, dc64, out, spread);
                if (m == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(1024), 0, 0, d16, c32, dc64, out, spread);
                if (m == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(1024), 0, 0, d16, c32, dc64, out, spread);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms; (void)hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            const double steps_per_cu = (double)blocks * 16 * kSteps / 256;
            printf("spread %d px  %-10s  %.3f ms  %.2f ns per wave-step per CU\n", spread, names[m], best,
                   best * 1e6 / steps_per_cu);
        }
    }
    return 0;
}
