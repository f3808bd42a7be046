// coherence_probe.hip -- one-off experiment (DESIGN.md §7 records the result).
// Kernel A: 2048 blocks, lane 0 of each does a returning device-scope atomicAdd on a counter and
// then plain-loads the counter's cache line (as the hash allocator did).  Kernel B, launched
// right behind it on the same stream with no host sync, reads the counter three ways:
// scalar plain load, vector plain load, atomic RMW.  Repeated without host syncs.
#include <hip/hip_runtime.h>
#include <cstdio>

struct St { unsigned long long top, free_, cursor, ovf; };

__global__ void alloc_like(St* st, unsigned long long* sink) {
    if (threadIdx.x == 0) {
        const unsigned long long c = atomicAdd(&st->cursor, 1ull);
        const unsigned long long nf = st->free_;
        const unsigned long long t = st->top;
        if (c + nf + t == 0xdeadbeefull) sink[0] = c;
    }
}

__global__ void commit_like(St* st, unsigned long long* out, int it) {
    const unsigned long long s = st->cursor;                                      // uniform: s_load
    const unsigned long long v = ((volatile St*)st)[threadIdx.x & 0].cursor;      // vector load
    const unsigned long long a = atomicAdd(&st->cursor, 0ull);                    // memory-side RMW
    out[3 * it + 0] = s;
    out[3 * it + 1] = v;
    out[3 * it + 2] = a;
    st->cursor = 0;  // like k_commit
}

__global__ void write_rows(int* a, int round) { a[blockIdx.x * 64 + threadIdx.x] = round * 100000 + blockIdx.x; }

__global__ void check_rows(const int* a, int round, int nb, int* bad) {
    const int src = (blockIdx.x + 3) % nb;
    const int v = a[src * 64 + threadIdx.x];
    if (v != round * 100000 + src) atomicAdd(bad, 1);
}

int main() {
    const int NB = 2048, IT = 200;
    St* st;
    unsigned long long *sink, *out;
    int *rows, *bad;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipMalloc(&st, sizeof(St));
    hipMalloc(&sink, 64);
    hipMalloc(&out, 3 * IT * 8);
    hipMalloc(&rows, NB * 64 * 4);
    hipMalloc(&bad, 4);
    hipMemset(st, 0, sizeof(St));
    hipMemset(bad, 0, 4);
    hipDeviceSynchronize();
    for (int it = 0; it < IT; ++it) {
        alloc_like<<<NB, 64, 0, s>>>(st, sink);
        commit_like<<<1, 1, 0, s>>>(st, out, it);
    }
    unsigned long long h[3 * IT];
    hipStreamSynchronize(s);
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    int bad_s = 0, bad_v = 0, bad_a = 0;
    for (int it = 0; it < IT; ++it) {
        bad_s += h[3 * it] != NB;
        bad_v += h[3 * it + 1] != NB;
        bad_a += h[3 * it + 2] != NB;
    }
    printf("counter after atomics, next kernel, no host sync: wrong scalar %d vector %d rmw %d of %d\n",
           bad_s, bad_v, bad_a, IT);
    printf("first: %llu %llu %llu\n", h[0], h[1], h[2]);
    int nbad = 0;
    write_rows<<<NB, 64, 0, s>>>(rows, 0);
    for (int r = 1; r <= 100; ++r) {
        check_rows<<<NB, 64, 0, s>>>(rows, r - 1, NB, bad);
        write_rows<<<NB, 64, 0, s>>>(rows, r);
        check_rows<<<NB, 64, 0, s>>>(rows, r, NB, bad);
    }
    hipStreamSynchronize(s);
    hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
    printf("plain store -> next-kernel plain load, cross block, no host sync: %d stale \n", nbad);
    printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
