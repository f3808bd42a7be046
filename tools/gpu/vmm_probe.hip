// vmm_probe.hip -- does the HIP virtual-memory API on this box support a reserved range backed by
// several physical chunks mapped one after another (the hash pool's growth, csrc/tsdf_hash.hip
// VArray)?  Prints the granularities and the result of each step; writes and reads every chunk.
//   hipcc -O2 --offload-arch=gfx950 tools/gpu/vmm_probe.hip -o /tmp/vmm_probe && /tmp/vmm_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(unsigned* p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (unsigned)i;
}
__global__ void k_check(const unsigned* p, size_t n, unsigned v, unsigned* bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != v + (unsigned)i) atomicAdd(bad, 1u);
}

int main() {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gmin = 0, grec = 0;
    printf("granularity min: %s %zu\n", hipGetErrorString(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum)), gmin);
    printf("granularity rec: %s %zu\n", hipGetErrorString(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended)), grec);
    for (size_t g : {gmin, grec}) {
        if (!g) continue;
        void* base = nullptr;
        const size_t total = 64 * g;
        hipError_t e = hipMemAddressReserve(&base, total, g, nullptr, 0);
        printf("[g=%zu] reserve %zu: %s\n", g, total, hipGetErrorString(e));
        if (e != hipSuccess) { (void)hipGetLastError(); continue; }
        size_t off = 0;
        const size_t sizes[3] = {3 * g, 5 * g, 8 * g};
        int ok = 1;
        for (size_t sz : sizes) {
            hipMemGenericAllocationHandle_t h;
            e = hipMemCreate(&h, sz, &prop, 0);
            printf("[g=%zu] create %zu: %s\n", g, sz, hipGetErrorString(e));
            if (e != hipSuccess) { ok = 0; break; }
            e = hipMemMap((char*)base + off, sz, 0, h, 0);
            printf("[g=%zu] map at +%zu: %s\n", g, off, hipGetErrorString(e));
            if (e != hipSuccess) { ok = 0; break; }
            hipMemAccessDesc acc{};
            acc.location = prop.location;
            acc.flags = hipMemAccessFlagsProtReadWrite;
            e = hipMemSetAccess((char*)base + off, sz, &acc, 1);
            printf("[g=%zu] access: %s\n", g, hipGetErrorString(e));
            if (e != hipSuccess) { ok = 0; break; }
            off += sz;
        }
        (void)hipGetLastError();
        if (ok) {
            unsigned* bad;
            (void)hipMalloc(&bad, 4);
            (void)hipMemset(bad, 0, 4);
            const size_t n = off / 4;
            hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (unsigned*)base, n, 7u);
            hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, (const unsigned*)base, n, 7u, bad);
            unsigned hb = 0;
            (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
            printf("[g=%zu] %zu bytes over 3 chunks written/read: %u mismatches (%s)\n", g, off, hb,
                   hipGetErrorString(hipGetLastError()));
        }
    }
    return 0;
}
