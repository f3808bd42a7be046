// dequeue_probe.hip -- (1) which XCC_ID values blocks read (s_getreg HW_REG_XCC_ID), and
// (2) returning device-scope atomicAdd dequeue throughput with 1 head vs 8 heads at several
// spacings, every wave of a 256-CU x 16-wave grid pulling until N tickets are handed out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_xcc(int* out) {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
}

__global__ void k_deq(unsigned* heads, int stride_words, int nheads, unsigned n_per_head, unsigned long long* sink) {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    const int h = (x & 7) % nheads;
    const int lane = threadIdx.x & 63;
    unsigned long long acc = 0;
    for (;;) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(heads + (size_t)h * stride_words, 1u);
        t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
        if (t >= n_per_head) break;
        acc += t;
    }
    if (lane == 0 && acc == 12345678901ull) sink[0] = acc;
}

int main() {
    int* dx;
    hipMalloc(&dx, 4096 * sizeof(int));
    hipLaunchKernelGGL(k_xcc, dim3(4096), dim3(64), 0, 0, dx);
    std::vector<int> hx(4096);
    hipMemcpy(hx.data(), dx, 4096 * sizeof(int), hipMemcpyDeviceToHost);
    int cnt[16] = {0};
    for (int v : hx) cnt[v & 15]++;
    printf("XCC_ID histogram over 4096 blocks:");
    for (int i = 0; i < 16; ++i) printf(" %d:%d", i, cnt[i]);
    printf("\nfirst 16 blocks:");
    for (int i = 0; i < 16; ++i) printf(" %d", hx[i]);
    printf("\n");
    unsigned* heads;
    const size_t maxw = 8 * 65536;
    hipMalloc(&heads, maxw * sizeof(unsigned));
    unsigned long long* sink;
    hipMalloc(&sink, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Cfg { int nheads, stride; } cfgs[] = {{1, 16}, {8, 16}, {8, 64}, {8, 256}, {8, 1024}, {8, 16384}, {8, 65536}};
    const unsigned total = 200000;
    for (auto c : cfgs) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(heads, 0, maxw * sizeof(unsigned));
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_deq, dim3(1024), dim3(256), 0, 0, heads, c.stride, c.nheads, total / c.nheads, sink);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("heads %d stride %6d words: %u tickets in %.1f us = %.0f per us\n", c.nheads, c.stride, total,
               best * 1e3f, total / (best * 1e3f));
    }
    return 0;
}
