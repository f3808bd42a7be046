// vmm_remap_probe.hip -- does a piece mapped where an earlier piece was unmapped (the hash pool's
// trim, then growth) see its own memory?  Per round: map 4 pieces, fill them; unmap + release the
// top piece; allocate and fill an ordinary buffer (which may take the released pages); map a
// fresh piece at the same address and fill it; then check both.  A kernel write through a stale
// translation of the unmapped piece would land in the ordinary buffer.  Modes: 0 plain; 1 set
// access over the whole mapped range after the remap; 2 hipDeviceSynchronize + an ordinary
// hipMalloc/hipFree between unmap and remap.
//   hipcc -O2 --offload-arch=gfx950 tools/gpu/vmm_remap_probe.hip -o tools/gpu/vmm_remap_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(unsigned* p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v ^ (unsigned)i;
}
__global__ void k_check(const unsigned* p, size_t n, unsigned v, unsigned* bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != (v ^ (unsigned)i)) atomicAdd(bad, 1u);
}

static const size_t P = 8ull << 20;
static hipMemAllocationProp prop;

static hipError_t map_at(char* va, hipMemGenericAllocationHandle_t* h, size_t set_from, size_t set_len) {
    hipError_t e = hipMemCreate(h, P, &prop, 0);
    if (e == hipSuccess) e = hipMemMap(va, P, 0, *h, 0);
    if (e == hipSuccess) {
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess((char*)set_from, set_len, &acc, 1);
    }
    return e;
}

static unsigned check(const void* p, size_t bytes, unsigned v, unsigned* bad) {
    (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(512), dim3(256), 0, 0, (const unsigned*)p, bytes / 4, v, bad);
    unsigned hb = 0;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    return hb;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    unsigned* bad;
    (void)hipMalloc(&bad, 4);
    for (int mode = 0; mode < 3; ++mode) {
        int fails = 0;
        for (int round = 0; round < 12; ++round) {
            void* b = nullptr;
            if (hipMemAddressReserve(&b, 8 * P, 2u << 20, nullptr, 0) != hipSuccess) { printf("reserve failed\n"); return 1; }
            char* base = (char*)b;
            hipMemGenericAllocationHandle_t h[4];
            for (int k = 0; k < 4; ++k)
                if (map_at(base + k * P, &h[k], (size_t)(base + k * P), P) != hipSuccess) { printf("map failed\n"); return 1; }
            hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, 0, (unsigned*)base, 4 * P / 4, 0x1111u);
            (void)hipDeviceSynchronize();
            (void)hipMemUnmap(base + 3 * P, P);
            (void)hipMemRelease(h[3]);
            if (mode == 2) {
                (void)hipDeviceSynchronize();
                void* t;
                (void)hipMalloc(&t, 2u << 20);
                (void)hipFree(t);
            }
            unsigned* x;
            (void)hipMalloc(&x, 64ull << 20);
            hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, 0, x, (64ull << 20) / 4, 0x2222u);
            hipError_t e = mode == 1 ? map_at(base + 3 * P, &h[3], (size_t)base, 4 * P)
                                     : map_at(base + 3 * P, &h[3], (size_t)(base + 3 * P), P);
            if (e != hipSuccess) { printf("remap failed: %s\n", hipGetErrorString(e)); return 1; }
            hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, 0, (unsigned*)(base + 3 * P), P / 4, 0x3333u);
            (void)hipDeviceSynchronize();
            const unsigned bx = check(x, 64ull << 20, 0x2222u, bad);
            const unsigned bp = check(base + 3 * P, P, 0x3333u, bad);
            const unsigned bl = check(base, 3 * P, 0x1111u, bad);
            // the remapped piece read by a copy engine (its own translation) against what the kernel wrote
            static unsigned hostbuf[(8u << 20) / 4];
            (void)hipMemcpy(hostbuf, base + 3 * P, P, hipMemcpyDeviceToHost);
            unsigned bc = 0;
            for (size_t i = 0; i < P / 4; ++i) bc += hostbuf[i] != (0x3333u ^ (unsigned)i);
            if (bx | bp | bl | bc) ++fails;
            printf("mode %d round %2d: other buffer %u, remapped piece %u (copy engine %u), kept pieces %u\n", mode, round, bx, bp, bc, bl);
            (void)hipFree(x);
            for (int k = 0; k < 4; ++k) {
                (void)hipMemUnmap(base + k * P, P);
                (void)hipMemRelease(h[k]);
            }
            (void)hipMemAddressFree(b, 8 * P);
        }
        printf("mode %d: %d of 12 rounds wrong\n", mode, fails);
    }
    return 0;
}
