// Contended device-scope atomics on MI355X: n waves (spread over the GPU, one per workgroup of 64
// threads, `spacing` waves of work between them) each do one atomicAdd on a counter; the counter
// is one address (mode 0), one per XCD (mode 1: blockIdx % 8), or one per workgroup (mode 2).
// Prints the kernel time for each mode (hipEvent), the cost the hash's pool_alloc would pay if
// every inserting wave hit one address.
//   hipcc --offload-arch=gfx950 -O2 tools/gpu/atomic_probe.hip -o /tmp/atomic_probe && /tmp/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_atomics(unsigned long long* ctr, int mode, int reps, unsigned long long* sink) {
    if (threadIdx.x != 0) return;
    const int slot = mode == 0 ? 0 : mode == 1 ? (blockIdx.x & 7) * 16 : (blockIdx.x % 4096) * 16;
    unsigned long long acc = 0;
    for (int r = 0; r < reps; ++r) acc += atomicAdd(ctr + slot, 1ull);
    if (acc == 0xFFFFFFFFFFFFull) sink[0] = acc;
}

int main() {
    unsigned long long *ctr, *sink;
    hipMalloc(&ctr, sizeof(unsigned long long) * 4096 * 16);
    hipMalloc(&sink, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {512, 4096};
    for (int g : grids)
        for (int reps : {1, 8})
            for (int mode = 0; mode < 3; ++mode) {
                hipMemset(ctr, 0, sizeof(unsigned long long) * 4096 * 16);
                hipLaunchKernelGGL(k_atomics, dim3(g), dim3(64), 0, 0, ctr, mode, reps, sink);  // warm
                hipDeviceSynchronize();
                float best = 1e9f;
                for (int t = 0; t < 5; ++t) {
                    hipEventRecord(a);
                    hipLaunchKernelGGL(k_atomics, dim3(g), dim3(64), 0, 0, ctr, mode, reps, sink);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    best = ms < best ? ms : best;
                }
                printf("{\"waves\": %d, \"atomics_per_wave\": %d, \"mode\": \"%s\", \"kernel_us\": %.2f, \"ns_per_atomic\": %.2f}\n",
                       g, reps, mode == 0 ? "one address" : mode == 1 ? "one per XCD" : "one per wave",
                       best * 1e3, best * 1e6 / (g * reps));
            }
    return 0;
}
