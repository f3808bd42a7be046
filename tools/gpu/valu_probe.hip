// valu_probe.hip -- issue cost of the VALU instructions the integrate kernel is made of, on
// gfx950: 8 independent chains per lane, W waves per SIMD, shader cycles from s_memtime.
// Prints cycles per wave-instruction per SIMD (throughput, all waves of the SIMD issuing).
//   hipcc -O3 --offload-arch=gfx950 tools/gpu/valu_probe.hip -o /tmp/valu_probe && /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kIters = 256;

#define BODY8(INS, T, C)                                                                        \
    asm volatile(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                 INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),      \
                   "+v"(a[6]), "+v"(a[7])                                                      \
                 : C(b))
#define BODY8_1(INS)                                                                            \
    asm volatile(INS " %0, %0\n" INS " %1, %1\n" INS " %2, %2\n" INS " %3, %3\n" INS " %4, %4\n" \
                 INS " %5, %5\n" INS " %6, %6\n" INS " %7, %7\n"                                \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),      \
                   "+v"(a[6]), "+v"(a[7]))
#define BODY8_3(INS)                                                                            \
    asm volatile(INS " %0, %0, %8, %8\n" INS " %1, %1, %8, %8\n" INS " %2, %2, %8, %8\n"         \
                 INS " %3, %3, %8, %8\n" INS " %4, %4, %8, %8\n" INS " %5, %5, %8, %8\n"         \
                 INS " %6, %6, %8, %8\n" INS " %7, %7, %8, %8\n"                                 \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),      \
                   "+v"(a[6]), "+v"(a[7])                                                      \
                 : "v"(b))

#define KERNEL(NAME, T, STMT)                                                                   \
    __global__ void NAME(T* out, long long* cyc, T b0) {                                        \
        T a[8];                                                                                 \
        for (int i = 0; i < 8; ++i) a[i] = (T)(threadIdx.x + i);                                \
        T b = b0;                                                                               \
        __syncthreads();                                                                        \
        const long long t0 = __builtin_amdgcn_s_memtime();                                      \
        for (int it = 0; it < kIters; ++it) { STMT; }                                           \
        const long long t1 = __builtin_amdgcn_s_memtime();                                      \
        T s = 0;                                                                                \
        for (int i = 0; i < 8; ++i) s += a[i];                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                         \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }

KERNEL(k_fma_f64, double, BODY8_3("v_fma_f64"))
KERNEL(k_add_f64, double, BODY8("v_add_f64", double, "v"))
KERNEL(k_mul_f64, double, BODY8("v_mul_f64", double, "v"))
KERNEL(k_rcp_f64, double, BODY8_1("v_rcp_f64"))
KERNEL(k_rndne_f64, double, BODY8_1("v_rndne_f64"))
KERNEL(k_fract_f64, double, BODY8_1("v_fract_f64"))
KERNEL(k_min_f64, double, BODY8("v_min_f64", double, "v"))
KERNEL(k_fma_f32, float, BODY8_3("v_fma_f32"))
KERNEL(k_add_f32, float, BODY8("v_add_f32", float, "v"))
KERNEL(k_rcp_f32, float, BODY8_1("v_rcp_f32"))
KERNEL(k_rndne_f32, float, BODY8_1("v_rndne_f32"))
KERNEL(k_pk_fma_f32, double, BODY8_3("v_pk_fma_f32"))
// conversions: 8 independent results per iteration from a source of the other width
#define BODYX(INS, SRC)                                                                          \
    asm volatile(INS " %0, %8\n" INS " %1, %8\n" INS " %2, %8\n" INS " %3, %8\n" INS " %4, %8\n"  \
                 INS " %5, %8\n" INS " %6, %8\n" INS " %7, %8\n"                                  \
                 : "=v"(a[0]), "=v"(a[1]), "=v"(a[2]), "=v"(a[3]), "=v"(a[4]), "=v"(a[5]),      \
                   "=v"(a[6]), "=v"(a[7])                                                      \
                 : "v"(SRC))
#define KERNELX(NAME, T, S, INS)                                                                \
    __global__ void NAME(T* out, long long* cyc, T b0) {                                        \
        T a[8];                                                                                 \
        S src = (S)(threadIdx.x + 1);                                                           \
        __syncthreads();                                                                        \
        const long long t0 = __builtin_amdgcn_s_memtime();                                      \
        for (int it = 0; it < kIters; ++it) {                                                   \
            BODYX(INS, src);                                                                    \
            asm volatile("" : "+v"(src));                                                       \
        }                                                                                       \
        const long long t1 = __builtin_amdgcn_s_memtime();                                      \
        T s = 0;                                                                                \
        for (int i = 0; i < 8; ++i) s += a[i];                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s + b0;                                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }
KERNEL(k_mov_b64, double, BODY8_1("v_mov_b64"))
KERNELX(k_cvt_f64_f32, double, float, "v_cvt_f64_f32")
KERNELX(k_cvt_f32_f64, float, double, "v_cvt_f32_f64")
KERNELX(k_cvt_f64_u32, double, unsigned, "v_cvt_f64_u32")
KERNELX(k_cvt_i32_f64, float, double, "v_cvt_i32_f64")
KERNEL(k_cvt_u32_f32, float, BODY8_1("v_cvt_u32_f32"))
KERNEL(k_cvt_ubyte1, float, BODY8_1("v_cvt_f32_ubyte1"))
KERNEL(k_mad_u24, float, BODY8_3("v_mad_u32_u24"))
KERNEL(k_pk_mul_f32, double, BODY8("v_pk_mul_f32", double, "v"))

typedef void (*kd)(double*, long long*, double);
typedef void (*kf)(float*, long long*, float);

template <typename T, typename K>
void run(const char* name, K k, int waves_per_simd) {
    const int cus = 256, wg = 64 * 4 * waves_per_simd;  // one workgroup per CU, W waves per SIMD
    T* out;
    long long* cyc;
    hipMalloc(&out, sizeof(T) * cus * wg);
    hipMalloc(&cyc, sizeof(long long) * cus * wg / 64);
    hipLaunchKernelGGL(k, dim3(cus), dim3(wg), 0, 0, out, cyc, (T)1.0000001);
    hipLaunchKernelGGL(k, dim3(cus), dim3(wg), 0, 0, out, cyc, (T)1.0000001);
    hipDeviceSynchronize();
    std::vector<long long> h(cus * wg / 64);
    hipMemcpy(h.data(), cyc, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    double mean = 0;
    for (long long c : h) mean += (double)c;
    mean /= h.size();
    // s_memtime counts at a constant 100 MHz on some parts; report raw ticks per instruction too
    const double per = mean / (kIters * 8.0) / waves_per_simd;
    printf("%-14s W=%d  ticks/wave-instr/SIMD %.3f\n", name, waves_per_simd, per);
    hipFree(out);
    hipFree(cyc);
}

// v_cvt_pk_u8_f32 rounding: every quarter value in [-2, 260] against rint + clamp
__global__ void k_pk_u8(unsigned* bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float x = -2.0f + 0.25f * (float)i;
    if (x > 260.0f) return;
    unsigned r;
    asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, 0" : "=v"(r) : "v"(x));
    const float e = fminf(fmaxf(rintf(x), 0.0f), 255.0f);
    if ((r & 0xFF) != (unsigned)e) atomicAdd(bad, 1u);
}

int main() {
    {
        unsigned* bad;
        hipMalloc(&bad, 4);
        hipMemset(bad, 0, 4);
        hipLaunchKernelGGL(k_pk_u8, dim3(8), dim3(256), 0, 0, bad);
        unsigned h = 0;
        hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
        printf("v_cvt_pk_u8_f32 vs rint+clamp: %u mismatches of 1049 quarter values\n", h);
        hipFree(bad);
    }
    for (int w : {1, 4}) {
        run<double>("v_fma_f64", (kd)k_fma_f64, w);
        run<double>("v_add_f64", (kd)k_add_f64, w);
        run<double>("v_mul_f64", (kd)k_mul_f64, w);
        run<double>("v_rcp_f64", (kd)k_rcp_f64, w);
        run<double>("v_rndne_f64", (kd)k_rndne_f64, w);
        run<double>("v_fract_f64", (kd)k_fract_f64, w);
        run<double>("v_min_f64", (kd)k_min_f64, w);
        run<float>("v_fma_f32", (kf)k_fma_f32, w);
        run<float>("v_add_f32", (kf)k_add_f32, w);
        run<float>("v_rcp_f32", (kf)k_rcp_f32, w);
        run<float>("v_rndne_f32", (kf)k_rndne_f32, w);
        run<double>("v_pk_fma_f32", (kd)k_pk_fma_f32, w);
        run<double>("v_pk_mul_f32", (kd)k_pk_mul_f32, w);
        run<double>("v_mov_b64", (kd)k_mov_b64, w);
        run<double>("v_cvt_f64_f32", (kd)k_cvt_f64_f32, w);
        run<float>("v_cvt_f32_f64", (kf)k_cvt_f32_f64, w);
        run<double>("v_cvt_f64_u32", (kd)k_cvt_f64_u32, w);
        run<float>("v_cvt_i32_f64", (kf)k_cvt_i32_f64, w);
        run<float>("v_cvt_u32_f32", (kf)k_cvt_u32_f32, w);
        run<float>("v_cvt_f32_ubyte1", (kf)k_cvt_ubyte1, w);
        run<float>("v_mad_u32_u24", (kf)k_mad_u24, w);
    }
    return 0;
}
