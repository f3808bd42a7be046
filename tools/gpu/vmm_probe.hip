// vmm_probe.hip -- the HIP virtual-memory API on this box with the hash pool's growth pattern
// (csrc/tsdf_hash.hip VArray): a reserved range backed by chunks mapped one after another.
// Prints the granularities and the result of each step for several (reserve alignment, chunk
// rounding) choices; writes and reads every mapped byte.
//   hipcc -O2 --offload-arch=gfx950 tools/gpu/vmm_probe.hip -o tools/gpu/vmm_probe && tools/gpu/vmm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_fill(unsigned* p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (unsigned)i;
}
__global__ void k_check(const unsigned* p, size_t n, unsigned v, unsigned* bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != v + (unsigned)i) atomicAdd(bad, 1u);
}

// piece: 0 = 8 MB then 32 MB pieces (the library), else a fixed piece size; whole: set access
// over everything mapped so far instead of over the new chunk only
static int trial(size_t align, size_t round, size_t piece, bool whole, const std::vector<size_t>& wants, const hipMemAllocationProp& prop) {
    void* base = nullptr;
    const size_t total = 1ull << 30;
    hipError_t e = hipMemAddressReserve(&base, total, align, nullptr, 0);
    printf("align %zu round %zu piece %zu whole %d: reserve %s base %% 2MB = %zu\n", align, round, piece, (int)whole, hipGetErrorString(e),
           (size_t)base % (2u << 20));
    if (e != hipSuccess) return (void)hipGetLastError(), 0;
    size_t mapped = 0;
    int ok = 1;
    for (size_t want : wants) {
        want = (want + round - 1) / round * round;
        while (ok && mapped < want) {
            const size_t sz = piece ? std::min(piece, want - mapped) : std::min<size_t>(32ull << 20, want - mapped);
            hipMemGenericAllocationHandle_t h;
            e = hipMemCreate(&h, sz, &prop, 0);
            if (e == hipSuccess) e = hipMemMap((char*)base + mapped, sz, 0, h, 0);
            if (e == hipSuccess) {
                hipMemAccessDesc acc{};
                acc.location = prop.location;
                acc.flags = hipMemAccessFlagsProtReadWrite;
                e = whole ? hipMemSetAccess(base, mapped + sz, &acc, 1) : hipMemSetAccess((char*)base + mapped, sz, &acc, 1);
            }
            printf("  chunk %zu at +%zu: %s\n", sz, mapped, hipGetErrorString(e));
            if (e != hipSuccess) ok = 0;
            else mapped += sz;
        }
    }
    (void)hipGetLastError();
    if (ok) {
        unsigned* bad;
        (void)hipMalloc(&bad, 4);
        (void)hipMemset(bad, 0, 4);
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (unsigned*)base, mapped / 4, 7u);
        hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, (const unsigned*)base, mapped / 4, 7u, bad);
        unsigned hb = 0;
        (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        printf("  %zu bytes written/read: %u mismatches (%s)\n", mapped, hb, hipGetErrorString(hipGetLastError()));
    }
    return ok;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gmin = 0, grec = 0;
    printf("granularity min: %s %zu\n", hipGetErrorString(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum)), gmin);
    printf("granularity rec: %s %zu\n", hipGetErrorString(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended)), grec);
    // the pool's pattern: 8 MB at create, then growth to 90.6 MB and 300 MB (2 KB blocks)
    const std::vector<size_t> wants = {8ull << 20, 44242ull * 2048, 150000ull * 2048};
    const size_t MB2 = 2u << 20;
    for (int rep = 0; rep < 2; ++rep) {
        trial(MB2, grec, 0, false, wants, prop);
        trial(MB2, grec, 0, true, wants, prop);
        trial(MB2, MB2, 2ull << 20, false, wants, prop);
        trial(MB2, MB2, 8ull << 20, false, wants, prop);
        trial(MB2, 32ull << 20, 32ull << 20, false, wants, prop);
        trial(MB2, 32ull << 20, 32ull << 20, true, wants, prop);
    }
    return 0;
}
