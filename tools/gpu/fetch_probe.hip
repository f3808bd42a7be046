// fetch_probe.hip -- what the L2's memory-side read counters tally for the integrate kernel's access
// classes on gfx950, on launches whose byte counts are known exactly.  Run under
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
//             --kernel-trace -- ./tools/gpu/fetch_probe
// (and a FETCH_SIZE pass): each kernel's request counts by size against the bytes it must fetch.
//   hipcc -O3 --offload-arch=gfx950 tools/gpu/fetch_probe.hip -o tools/gpu/fetch_probe
// Kernels (every buffer first flushed out of the caches by streaming a 1 GB buffer through them):
//   k_stream16   16-B/lane coalesced reads of a 256 MB buffer (the brick-state loads' form)
//   k_gather2    one 2-byte load per 128-B line, every line of a 256 MB buffer once (depth texels
//                that miss every cache: what one L2 line fill tallies)
//   k_gather2x2  two 2-byte loads per 128-B line, at bytes 0 and 64, by the same wave back to back
//                (is a fill 128 B or a 64-B sector?)
//   k_gather4    one 4-byte load per 128-B line (the RGB8 gathers' dword loads)
//   k_resident   2-byte gathers spread over a 48 MB set (a launch's 32 frames of u16 + RGB8) that
//                was read just before, so it sits in the Infinity Cache but not in the 4 MB L2s:
//                the integrate's gather fills, each counted once per L2 fill
// Prints each kernel's bytes that must be fetched; the profile gives the requests.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBig = 256ull << 20;    // 256 MB: the gather / stream buffers
constexpr size_t kFlush = 1024ull << 20; // 1 GB flush buffer (> the 256 MB Infinity Cache)
constexpr size_t kRes = 48ull << 20;     // 48 MB resident set

__global__ void k_flush(const float4* p, size_t n, float* out) {
    float acc = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;  // (never: keeps the loads)
}

__global__ void k_stream16(const float4* p, size_t n, float* out) {
    float acc = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

// lane i of the grid reads line i (a permutation keeps neighbouring lanes off neighbouring lines;
// 40507 is odd and not a multiple of 3: a bijection for 2^k and 3 * 2^k lines)
__device__ inline size_t line_of(size_t i, size_t n_lines) { return (i * 40507ull) % n_lines; }

__global__ void k_gather2(const unsigned short* p, size_t n_lines, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_lines; i += (size_t)gridDim.x * blockDim.x)
        acc += p[line_of(i, n_lines) * 64];
    if (acc == 0xdeadbeefu) out[0] = acc;
}

__global__ void k_gather2x2(const unsigned short* p, size_t n_lines, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_lines; i += (size_t)gridDim.x * blockDim.x) {
        const size_t l = line_of(i, n_lines) * 64;
        acc += p[l];
        acc += p[l + 32];  // byte 64 of the same line (a second load instruction)
    }
    if (acc == 0xdeadbeefu) out[0] = acc;
}

__global__ void k_gather4(const unsigned* p, size_t n_lines, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_lines; i += (size_t)gridDim.x * blockDim.x)
        acc += p[line_of(i, n_lines) * 32];
    if (acc == 0xdeadbeefu) out[0] = acc;
}

// each line of the resident set gathered once (2 bytes at a random offset inside it)
__global__ void k_resident(const unsigned short* p, size_t n_lines, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_lines; i += (size_t)gridDim.x * blockDim.x)
        acc += p[line_of(i, n_lines) * 64 + (i * 7) % 64];
    if (acc == 0xdeadbeefu) out[0] = acc;
}

int main() {
    char *big, *flush, *res;
    float* out;
    if (hipMalloc(&big, kBig) != hipSuccess || hipMalloc(&flush, kFlush) != hipSuccess ||
        hipMalloc(&res, kRes) != hipSuccess || hipMalloc(&out, 256) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(big, 1, kBig);
    (void)hipMemset(flush, 2, kFlush);
    (void)hipMemset(res, 3, kRes);
    (void)hipDeviceSynchronize();
    const dim3 g(256 * 8), b(256);
    auto flush_caches = [&] {
        hipLaunchKernelGGL(k_flush, g, b, 0, 0, (const float4*)flush, kFlush / 16, out);
        (void)hipDeviceSynchronize();
    };
    const size_t lines = kBig / 128;
    flush_caches();
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const float4*)big, kBig / 16, out);
    (void)hipDeviceSynchronize();
    printf("k_stream16   must fetch %zu B (%zu x 128-B lines)\n", kBig, lines);
    flush_caches();
    hipLaunchKernelGGL(k_gather2, g, b, 0, 0, (const unsigned short*)big, lines, (unsigned*)out);
    (void)hipDeviceSynchronize();
    printf("k_gather2    touches %zu distinct 128-B lines once (2 B used of each)\n", lines);
    flush_caches();
    hipLaunchKernelGGL(k_gather2x2, g, b, 0, 0, (const unsigned short*)big, lines, (unsigned*)out);
    (void)hipDeviceSynchronize();
    printf("k_gather2x2  touches %zu distinct 128-B lines, bytes 0 and 64 of each\n", lines);
    flush_caches();
    hipLaunchKernelGGL(k_gather4, g, b, 0, 0, (const unsigned*)big, lines, (unsigned*)out);
    (void)hipDeviceSynchronize();
    printf("k_gather4    touches %zu distinct 128-B lines once (4 B used of each)\n", lines);
    flush_caches();
    const size_t rl = kRes / 128;
    // warm the resident set into the Infinity Cache (and then push it out of the 4 MB L2s with a
    // 32 MB stream that itself stays far below the Infinity Cache)
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const float4*)res, kRes / 16, out);
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const float4*)big, (32ull << 20) / 16, out);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_resident, g, b, 0, 0, (const unsigned short*)res, rl, (unsigned*)out);
    (void)hipDeviceSynchronize();
    printf("k_resident   touches %zu distinct 128-B lines of a 48 MB Infinity-Cache-resident set once\n", rl);
    (void)hipFree(big);
    (void)hipFree(flush);
    (void)hipFree(res);
    (void)hipFree(out);
    return 0;
}
