// kernarg_probe.hip -- largest by-value kernel argument the HIP runtime accepts on gfx950
// (does a 3-batch pipeline launch fit in kernel arguments?).  Prints per size: launch status and
// whether the kernel saw every byte.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
struct Blob { unsigned w[N / 4]; };

template <int N>
__global__ void k_sum(Blob<N> b, unsigned long long* out) {
    unsigned long long s = 0;
    for (int i = threadIdx.x; i < N / 4; i += blockDim.x) s += b.w[i];
    atomicAdd(out, s);
}

template <int N>
void run() {
    Blob<N> b;
    unsigned long long want = 0;
    for (int i = 0; i < N / 4; ++i) { b.w[i] = (unsigned)(i * 2654435761u) >> 8; want += b.w[i]; }
    unsigned long long* d;
    hipMalloc(&d, 8);
    hipMemset(d, 0, 8);
    hipLaunchKernelGGL(k_sum<N>, dim3(1), dim3(256), 0, 0, b, d);
    hipError_t e = hipGetLastError();
    hipError_t e2 = hipDeviceSynchronize();
    unsigned long long got = 0;
    hipMemcpy(&got, d, 8, hipMemcpyDeviceToHost);
    printf("%6d bytes: launch %s, sync %s, %s\n", N, hipGetErrorString(e), hipGetErrorString(e2),
           got == want ? "sum OK" : "sum WRONG");
    hipFree(d);
}

int main() {
    run<2048>();
    run<4096>();
    run<6144>();
    run<8192>();
    run<12288>();
    run<16384>();
    run<24576>();
    run<32768>();
    run<40960>();
    run<49152>();
    run<65536>();
    return 0;
}
