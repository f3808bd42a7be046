// tsdf_common.hip -- errors, device discovery, frame staging, pyramid launch, profiling and
// the bulk hash_function entry point of the C-ABI (include/tsdf_hip.h).
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "tsdf_host.h"

namespace tsdf {

static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

PyrLayout pyr_layout(int H, int W) {
    PyrLayout l{};
    int off = 0;
    for (int L = 1; L <= kPyrLevels; ++L) {
        l.w[L] = (W + (1 << L) - 1) >> L;
        l.h[L] = (H + (1 << L) - 1) >> L;
        l.off[L] = off;
        off += l.w[L] * l.h[L];
    }
    l.total = off;
    return l;
}

// Timing-only events: no system-scope fence when they complete (hip_runtime_api.h documents
// hipEventDisableSystemFence for exactly this use), so recording them does not add a cache
// writeback between the kernels they bracket.  TSDF_PROF_EVFLAGS overrides (A/B).
static int new_timing_event(hipEvent_t* e) {
    const char* ef = getenv("TSDF_PROF_EVFLAGS");
    const unsigned fl = ef ? (unsigned)strtoul(ef, nullptr, 0) : (unsigned)hipEventDisableSystemFence;
    TSDF_HIP(hipEventCreateWithFlags(e, fl));
    return TSDF_OK;
}

int Profiler::begin(hipStream_t s, hipEvent_t* e0) {
    *e0 = nullptr;
    if (!on) return TSDF_OK;
    if (spare.empty()) {
        hipEvent_t e;
        TSDF_TRY(new_timing_event(&e));
        spare.push_back(e);
    }
    *e0 = spare.back();
    spare.pop_back();
    TSDF_HIP(hipEventRecord(*e0, s));
    return TSDF_OK;
}

int Profiler::end(hipStream_t s, hipEvent_t e0) {
    if (!on || !e0) return TSDF_OK;
    if (spare.empty()) {
        hipEvent_t e;
        TSDF_TRY(new_timing_event(&e));
        spare.push_back(e);
    }
    hipEvent_t e1 = spare.back();
    spare.pop_back();
    TSDF_HIP(hipEventRecord(e1, s));
    pending.emplace_back(e0, e1);
    return TSDF_OK;
}

int Profiler::collect() {
    for (auto& pr : pending) {
        TSDF_HIP(hipEventSynchronize(pr.second));
        float t = 0.0f;
        TSDF_HIP(hipEventElapsedTime(&t, pr.first, pr.second));
        ms += t;
        ++launches;
        spare.push_back(pr.first);
        spare.push_back(pr.second);
    }
    pending.clear();
    return TSDF_OK;
}

void Profiler::release() {
    for (auto& pr : pending) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (auto e : spare) (void)hipEventDestroy(e);
    pending.clear();
    spare.clear();
}

__global__ void k_zero_u64(unsigned long long* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0ull;
}

namespace {
// Vol::canon check over the first n voxels of the brick pool: weights integers >= 0, colours
// canonical (the state integrate writes); any other value clears the flag (k_set / import).
__global__ void k_check_canon(const float* __restrict__ w, const float* __restrict__ c, size_t n, int* bad) {
    bool ok = true;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float wi = w[i], ci = c[i];
        ok = ok && wi >= 0.0f && wi == truncf(wi) && ci >= 0.0f && ci < 16777216.0f && ci == truncf(ci);
    }
    if (__ballot(!ok) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

__global__ void k_fill_rcp(double* r) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < kRcpBig) r[i] = 1.0 / (double)i;  // IEEE division: RN(1/i) (r[0] = inf, unused)
}
}  // namespace

int Base::init(int dev, const int64_t dims[3], const int64_t off[3], const float origin[3],
               double vs, double trunc) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(TSDF_E_NODEV, "no HIP device visible");
    if (dev < 0 || dev >= ndev) return set_error(TSDF_E_ARG, "device %d out of range [0,%d)", dev, ndev);
    device = dev;
    TSDF_HIP(hipSetDevice(device));
    if (const char* e = getenv("TSDF_CULL_G")) cull_g = atoi(e);  // A/B override (Base::cull_per_wg)
    for (int a = 0; a < 3; ++a) {
        const int64_t o = off ? off[a] : 0;
        if (dims[a] <= 0 || o < 0 || dims[a] + o > (1 << 24))
            return set_error(TSDF_E_ARG, "dims/index_offset out of range on axis %d (%lld + %lld)", a,
                             (long long)dims[a], (long long)o);
        vol.dims[a] = (int)dims[a];
        vol.off[a] = (int)o;
        vol.nb[a] = (int)((dims[a] + kBrickEdge - 1) / kBrickEdge);
        vol.origin[a] = origin[a];
    }
    if (!(vs > 0.0) || !(trunc > 0.0)) return set_error(TSDF_E_ARG, "voxel_size and trunc must be > 0");
    vol.vs = vs;
    vol.trunc = trunc;
    vol.rtrunc = 1.0 / trunc;  // IEEE division: RN(1/trunc)
    vol.xstride = vol.xodd = kBrickEdge;
    vol.sb[0] = vol.sb[1] = vol.sb[2] = 2;  // 4x4x4-brick superbricks
    vol.shard = 0;
    vol.n_shards = 1;
    vol.canon = 1;  // a fresh state (1, 0, 0) everywhere
    n_bricks = (long long)vol.nb[0] * vol.nb[1] * vol.nb[2];
    if (n_bricks >= (1ll << 24)) return set_error(TSDF_E_ARG, "too many bricks (%lld >= 2^24)", n_bricks);
    TSDF_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    TSDF_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    for (int k = 0; k < kSlots; ++k) {
        TSDF_HIP(hipEventCreateWithFlags(&ev_copied[k], hipEventDisableTiming));
        TSDF_HIP(hipEventCreateWithFlags(&ev_free[k], hipEventDisableTiming));
        TSDF_HIP(hipEventRecord(ev_free[k], stream));      // every slot starts free
        TSDF_HIP(hipEventRecord(ev_copied[k], cstream));
    }
    TSDF_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
    TSDF_HIP(hipMalloc(&rcp, sizeof(double) * kRcpBig));
    hipLaunchKernelGGL(k_fill_rcp, dim3((kRcpBig + 255) / 256), dim3(256), 0, stream, rcp);
    TSDF_HIP(hipGetLastError());
    vol.rcp = rcp;
    TSDF_HIP(hipMalloc(&stats, sizeof(unsigned long long) * kNStat * kStatSpread));
    TSDF_HIP(hipMemsetAsync(stats, 0, sizeof(unsigned long long) * kNStat * kStatSpread, stream));
    return TSDF_OK;
}

// Frames per launch (the create functions call it once, after init): sizes the per-batch buffers,
// whose frame and cost-class dimension is the handle's batch (kFullBatch for a whole volume,
// kMaxBatch for a shard; TSDF_BATCH overrides), not the kernels' capacity kMaxBatch; then buffer
// set 0's list and counters.
int Base::set_batch(int want) {
    if (const char* e = getenv("TSDF_BATCH")) want = atoi(e);
    batch = want < 1 ? 1 : want > kMaxBatch ? kMaxBatch : want;
    defer_frames = batch < 8 ? batch : 8;
    if (const char* e = getenv("TSDF_DEFER_FRAMES")) defer_frames = atoi(e);
    defer_frames = defer_frames < 1 ? 1 : defer_frames > batch ? batch : defer_frames;
    if (const char* e = getenv("TSDF_DEFER_DMA_FRAMES")) dma_grain = atoi(e) < 1 ? 1 : atoi(e);
    if (const char* e = getenv("TSDF_RGB_DIRECT")) rgb_direct = atoi(e) != 0;  // (A/B, parity tests)
    if (const char* e = getenv("TSDF_TEXEL")) texel_mode = atoi(e) != 0;
    if (const char* e = getenv("TSDF_DEFER_MM")) defer_mm = atoi(e) != 0;
    if (list_set[0]) return TSDF_OK;
    TSDF_HIP(hipMalloc(&list_set[0], sizeof(ListEntry) * (size_t)n_bricks * batch));
    TSDF_HIP(hipMalloc(&count_set[0], sizeof(unsigned int) * kCountWords));
    TSDF_HIP(hipMemsetAsync(count_set[0], 0, sizeof(unsigned int) * kCountWords, stream));
    use_set(0);
    return TSDF_OK;
}

// Buffer sets 1..n-1 (lists and counters now; pyramids, RGBX and masks when a batch needs them).
int Base::use_sets(int n) {
    if (n <= n_sets) return TSDF_OK;
    TSDF_TRY(sync_all());
    for (int k = n_sets; k < n; ++k) {
        TSDF_HIP(hipMalloc(&list_set[k], sizeof(ListEntry) * (size_t)n_bricks * batch));
        TSDF_HIP(hipMalloc(&count_set[k], sizeof(unsigned int) * kCountWords));
        TSDF_HIP(hipMemsetAsync(count_set[k], 0, sizeof(unsigned int) * kCountWords, stream));
    }
    TSDF_HIP(hipStreamSynchronize(stream));
    n_sets = n;
    return TSDF_OK;
}

int Base::sync_all() {
    TSDF_HIP(hipStreamSynchronize(stream));
    if (cstream) TSDF_HIP(hipStreamSynchronize(cstream));
    return TSDF_OK;
}


int Base::ensure_pyr(int H, int W) {
    if (pyr_set[0] && H == pyr_H && W == pyr_W && pyr_set[n_sets - 1]) return TSDF_OK;
    TSDF_TRY(sync_all());
    for (int k = 0; k < kSets; ++k) {
        if (pyr_set[k]) TSDF_HIP(hipFree(pyr_set[k]));
        if (rgbx_set[k]) TSDF_HIP(hipFree(rgbx_set[k]));
        pyr_set[k] = nullptr;
        rgbx_set[k] = nullptr;
    }
    lay = pyr_layout(H, W);
    for (int k = 0; k < n_sets; ++k) {
        TSDF_HIP(hipMalloc(&pyr_set[k], sizeof(float) * (size_t)lay.total * batch));
        TSDF_HIP(hipMalloc(&rgbx_set[k], sizeof(unsigned) * 2 * (size_t)H * W * batch));  // (RGBX or texels)
    }
    pyr_H = H;
    pyr_W = W;
    use_set(cur_set);
    return TSDF_OK;
}

int check_frame_args(const void* depth, int dk, const void* color, int ck, int H, int W,
                     const double* K, const double* Tinv) {
    if (!depth || !color || !K || !Tinv) return set_error(TSDF_E_ARG, "null frame pointer");
    if (dk != TSDF_DEPTH_U16_MM && dk != TSDF_DEPTH_F64_M) return set_error(TSDF_E_ARG, "bad depth_kind %d", dk);
    if (ck != TSDF_COLOR_RGB8 && ck != TSDF_COLOR_F32) return set_error(TSDF_E_ARG, "bad color_kind %d", ck);
    // < 2^28 pixels and sides < 2^24: the integrate's gathers use 32-bit byte offsets (8-byte f64
    // depth texels) and a 24-bit multiply for v*W
    if (H <= 0 || W <= 0 || H >= (1 << 24) || W >= (1 << 24) || (long long)H * W >= (1ll << 28))
        return set_error(TSDF_E_ARG, "bad image size %dx%d", H, W);
    return TSDF_OK;
}

// Half-spaces n.q + d >= 0 (unit n, q = world point - camera centre) that contain every voxel
// the reference can update for this frame: z > 0 and -0.5 <= u < W - 0.5, -0.5 <= v < H - 0.5,
// each widened by one pixel (grid_fusion.py:273-277).  Camera-space plane (a, b, c, e) maps to
// world space through the rows of world_to_cam; relative to the camera centre its offset is
// small whatever the volume's distance from the world origin, so the cull's f32 test is exact to
// ~1e-6 m there too (a 1e-4 m slack covers it).
static void frustum_planes(Frame* fr, const double* T, int W, int H) {
    for (int a = 0; a < 3; ++a)  // camera centre: -R^T t of world_to_cam = [R | t]
        fr->eye[a] = -(T[a] * T[3] + T[4 + a] * T[7] + T[8 + a] * T[11]);
    const double cam[5][4] = {{0.0, 0.0, 1.0, 1e-4},
                              {fr->fx, 0.0, fr->cx + 1.5, 0.0},
                              {-fr->fx, 0.0, (double)W + 0.5 - fr->cx, 0.0},
                              {0.0, fr->fy, fr->cy + 1.5, 0.0},
                              {0.0, -fr->fy, (double)H + 0.5 - fr->cy, 0.0}};
    for (int i = 0; i < 5; ++i) {
        double n[3], d = cam[i][3];
        for (int a = 0; a < 3; ++a)
            n[a] = cam[i][0] * T[0 + a] + cam[i][1] * T[4 + a] + cam[i][2] * T[8 + a];
        d += cam[i][0] * T[3] + cam[i][1] * T[7] + cam[i][2] * T[11];
        d += n[0] * fr->eye[0] + n[1] * fr->eye[1] + n[2] * fr->eye[2];  // relative to the eye
        const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        const double s = len > 0.0 ? 1.0 / len : 0.0;
        for (int a = 0; a < 3; ++a) fr->planes[i][a] = (float)(n[a] * s);
        fr->planes[i][3] = (float)(d * s) + (len > 0.0 ? 1e-4f : 1.0f);  // slack for f32 rounding
    }
}

// f64 metres -> u16 millimetres where that is exact: every d must be RN(k / 1000) for an integer k
// in [0, 65535] -- what the demos' depth_im = png / 1000. holds -- checked by recomputing it as the
// kernels' u16 path does, fma(k, 0.001, k * C_LO) (exact for every u16, tools/check_depth_conversion.c),
// so the integrate sees the same metres either way; NaN, negatives, other values fail.  Returns
// whether all n did (dst is then complete).  -0.0 passes as 0, which every use of depth treats alike
// (depth > 0 and depth - z).
static inline bool depth_mm_range(unsigned short* dst, const double* src, size_t n) {
    unsigned bad = 0;
    for (size_t i = 0; i < n; ++i) {
        const double d = src[i];
        const double k = fmin(fmax(__builtin_rint(d * 1000.0), 0.0), 65535.0);  // (NaN -> 0)
        const double back = __builtin_fma(k, 0.001, k * -2.0858186326137145e-20);
        bad |= (unsigned)(back != d);
        dst[i] = (unsigned short)(int)k;
    }
    return bad == 0;
}
__attribute__((target("avx2,fma"))) static bool depth_mm_avx2(unsigned short* dst, const double* src, size_t n) {
    return depth_mm_range(dst, src, n);
}
static bool depth_mm_any(unsigned short* dst, const double* src, size_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    return avx2 ? depth_mm_avx2(dst, src, n) : depth_mm_range(dst, src, n);
}

// Host copies into the page-locked bounce slots (ingest and the deferred drop-in frames) by a
// persistent pool of copy threads: one 640x480 f64 depth frame is 2.4 MB, and a single-thread
// memcpy of it and its colour (~140 us) bounded the per-frame drop-in rate (6k frames/s; 10k
// with the pool); spawning threads per call cost more than it saved below 4 MB.  The caller copies
// one share itself.  A deferred frame is ONE job -- its depth (converted to u16 millimetres, or
// copied) and its colour, share by share -- so a frame costs one hand-off, and the workers spin on
// the job counter for a while after each job (TSDF_COPY_SPIN_US, 300 us by default) before they
// block: at the reference's one-call-per-frame rate (~100 us apart) they never sleep, so no frame
// waits for a thread to wake (round 5 handed each frame over twice through a condition variable,
// and the per-frame rate varied from 4.7k to 12.3k frames/s between boxes).
// TSDF_COPY_THREADS sets the pool size (0: copy on the calling thread).
namespace {
// Up to two parts, each split into the same number of shares: part a copies a_n bytes (kind 0) or
// converts a_n f64 depth values to u16 millimetres (kind 1, depth_mm_any); part b copies b_n bytes.
struct CopyJob {
    int a_kind = 0;
    char* a_dst = nullptr;
    const char* a_src = nullptr;
    size_t a_n = 0;
    char* b_dst = nullptr;
    const char* b_src = nullptr;
    size_t b_n = 0;
};

class CopyPool {
  public:
    static CopyPool& get() {
        static std::mutex mk;
        static CopyPool* pool = nullptr;
        std::lock_guard<std::mutex> g(mk);
        if (!pool || pool->pid_ != getpid()) pool = new CopyPool();  // (a forked child starts over;
        return *pool;                                                  //  the parent's pool is left)
    }
    void copy(void* dst, const void* src, size_t bytes) {
        if (workers_.empty() || bytes < (256u << 10)) {
            std::memcpy(dst, src, bytes);
            return;
        }
        CopyJob j;
        j.a_dst = (char*)dst, j.a_src = (const char*)src, j.a_n = bytes;
        run_job(j);
    }
    bool depth_mm(unsigned short* dst, const double* src, size_t n) {  // depth_mm_any over the pool
        if (workers_.empty() || n < (32u << 10)) return depth_mm_any(dst, src, n);
        CopyJob j;
        j.a_kind = 1, j.a_dst = (char*)dst, j.a_src = (const char*)src, j.a_n = n;
        return run_job(j);
    }
    // One deferred frame: its depth converted (convert: n_depth f64 values -> u16 at ddst; false
    // when a value is not exact millimetres) or copied (n_depth bytes), and its colour copied.
    bool frame(bool convert, void* ddst, const void* dsrc, size_t n_depth, void* cdst, const void* csrc,
               size_t c_bytes) {
        CopyJob j;
        j.a_kind = convert ? 1 : 0, j.a_dst = (char*)ddst, j.a_src = (const char*)dsrc, j.a_n = n_depth;
        j.b_dst = (char*)cdst, j.b_src = (const char*)csrc, j.b_n = c_bytes;
        if (workers_.empty()) return share(j, 0, 1);
        return run_job(j);
    }

  private:
    // the job's shares: share 0 on the calling thread, share k on worker k.  The job's flag (a value
    // that is not exact millimetres) belongs to the job: cleared and read under call_, so a
    // concurrent caller (handles driven from several threads: ctypes releases the GIL) can neither
    // clear another job's flag nor see it (round-5 advisor finding)
    bool run_job(const CopyJob& j) {
        std::lock_guard<std::mutex> call(call_);  // one job at a time through the pool
        job_ = j;
        bad_.store(0, std::memory_order_relaxed);
        left_.store((int)workers_.size(), std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_seq_cst);  // publishes job_
        if (sleepers_.load(std::memory_order_seq_cst) > 0) {
            std::lock_guard<std::mutex> g(m_);
            cv_.notify_all();
        }
        const bool ok0 = share(job_, 0, (int)workers_.size() + 1);
        while (left_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
        return ok0 && bad_.load(std::memory_order_relaxed) == 0;
    }
    static size_t chunk_of(size_t n, int parts) { return ((n + parts - 1) / parts + 63) / 64 * 64; }
    bool share(const CopyJob& j, int k, int parts) {
        bool ok = true;
        const size_t ca = chunk_of(j.a_n, parts), oa = (size_t)k * ca;
        if (oa < j.a_n) {
            const size_t len = std::min(ca, j.a_n - oa);
            if (j.a_kind == 0) std::memcpy(j.a_dst + oa, j.a_src + oa, len);
            else ok = depth_mm_any((unsigned short*)j.a_dst + oa, (const double*)j.a_src + oa, len);
        }
        const size_t cb = chunk_of(j.b_n, parts), ob = (size_t)k * cb;
        if (ob < j.b_n) std::memcpy(j.b_dst + ob, j.b_src + ob, std::min(cb, j.b_n - ob));
        return ok;
    }
    CopyPool() : pid_(getpid()) {
        // four workers where the host has the cores (two on small hosts): per-frame dense drop-in
        // on one MI355X box 13.2k frames/s with 2, 17.1k with 4, 18.9k with 6 -- and 12-13k with 8
        // or 10, past the box's CPU share with the workers spinning (tools/gpu/dropin_rate.py,
        // profiles/r06_dropin/); 4 keeps the margin
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        int n = (int)std::max(std::min(2u, hw / 2), std::min(4u, hw / 16));
        if (const char* e = getenv("TSDF_COPY_THREADS")) n = std::max(0, std::min(32, atoi(e)));
        if (const char* e = getenv("TSDF_COPY_SPIN_US")) spin_us_ = std::max(0, atoi(e));
        for (int i = 0; i < n; ++i) workers_.emplace_back([this, i] { run(i + 1); });
        for (auto& t : workers_) t.detach();  // live for the process
    }
    void run(int k) {
        unsigned long long seen = 0;
        for (;;) {
            // the next job: spin for spin_us_, then block until it is published
            const auto t0 = std::chrono::steady_clock::now();
            for (unsigned it = 1; gen_.load(std::memory_order_acquire) == seen; ++it) {
                __builtin_ia32_pause();
                if ((it & 255) == 0 &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
                    sleepers_.fetch_add(1, std::memory_order_seq_cst);
                    std::unique_lock<std::mutex> g(m_);
                    cv_.wait(g, [&] { return gen_.load(std::memory_order_seq_cst) != seen; });
                    sleepers_.fetch_sub(1, std::memory_order_seq_cst);
                }
            }
            seen = gen_.load(std::memory_order_acquire);
            const CopyJob j = job_;  // (written before gen_ moved; the caller waits for every share)
            if (!share(j, k, (int)workers_.size() + 1)) bad_.store(1, std::memory_order_relaxed);
            left_.fetch_sub(1, std::memory_order_release);
        }
    }
    pid_t pid_;
    std::vector<std::thread> workers_;
    std::mutex call_, m_;
    std::condition_variable cv_;
    CopyJob job_;
    std::atomic<unsigned long long> gen_{0};
    std::atomic<int> left_{0}, bad_{0}, sleepers_{0};
    int spin_us_ = 300;
};
}  // namespace

// (diagnostic / CPU tests, not in the header) the deferred frames' f64 -> u16 depth conversion:
// 1 if all n values converted exactly, else 0
extern "C" int tsdf_diag_depth_to_mm(const double* src, long long n, unsigned short* dst) {
    if (!src || !dst || n < 0) return set_error(TSDF_E_ARG, "bad arguments");
    return CopyPool::get().depth_mm(dst, src, (size_t)n) ? 1 : 0;
}

static void par_memcpy(void* dst, const void* src, size_t bytes) {
    if (bytes < (4u << 20)) {  // one frame (the drop-in's deferred frames): the pool
        CopyPool::get().copy(dst, src, bytes);
        return;
    }
    // whole batches (>= 4 MB): threads of their own -- measured faster than the pool here
    // (pcie_inclusive 8.5-8.9k frames/s against 7.0-7.3k through the pool)
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t nt = std::min<size_t>(8, hw ? hw : 1);
    std::vector<std::thread> th;
    const size_t chunk = (bytes + nt - 1) / nt;
    for (size_t i = 0; i < nt; ++i) {
        const size_t o = i * chunk;
        if (o >= bytes) break;
        th.emplace_back([=] { std::memcpy((char*)dst + o, (const char*)src + o, std::min(chunk, bytes - o)); });
    }
    for (auto& t : th) t.join();
}

int Base::prepare_batch(Batch* bt, const void* depth, int dk, const void* color, int ck, int H,
                        int W, const double K[9], const double* Tinv, const double* ow,
                        double ow_default, int flags, int first, int n, int slot) {
    // the caller selected this batch's buffer set (use_set); reallocation keeps the selection
    TSDF_TRY(ensure_pyr(H, W));
    const size_t npx = (size_t)H * W;
    const size_t dbytes = npx * (dk == TSDF_DEPTH_U16_MM ? 2 : 8);
    const size_t cbytes = npx * (ck == TSDF_COLOR_RGB8 ? 3 : 4);
    const char* d = (const char*)depth + dbytes * (size_t)first;
    const char* c = (const char*)color + cbytes * (size_t)first;
    if (!(flags & TSDF_DEVICE_PTRS)) {  // stage the batch's frames into staging slot `slot`
        if (prestaged >= 0) {  // deferred frames: already copied into bounce slot `prestaged`
            slot = prestaged;
        } else {
            TSDF_TRY(stage_alloc(dbytes, cbytes));
            // the bounce slot is free once its previous DMA has finished
            TSDF_HIP(hipEventSynchronize(ev_copied[slot]));
            par_memcpy(hst_depth[slot], d, dbytes * n);
            par_memcpy(hst_color[slot], c, cbytes * n);
        }
        // (deferred frames: the first pre_copied frames' DMA was issued while the batch filled)
        const size_t c0 = prestaged >= 0 ? (size_t)std::min(pre_copied, n) : 0;
        TSDF_HIP(hipStreamWaitEvent(cstream, ev_free[slot], 0));
        if (c0 < (size_t)n) {
            TSDF_HIP(hipMemcpyAsync((char*)st_depth[slot] + dbytes * c0, (const char*)hst_depth[slot] + dbytes * c0,
                                    dbytes * (n - c0), hipMemcpyHostToDevice, cstream));
            TSDF_HIP(hipMemcpyAsync((char*)st_color[slot] + cbytes * c0, (const char*)hst_color[slot] + cbytes * c0,
                                    cbytes * (n - c0), hipMemcpyHostToDevice, cstream));
        }
        TSDF_HIP(hipEventRecord(ev_copied[slot], cstream));
        TSDF_HIP(hipStreamWaitEvent(stream, ev_copied[slot], 0));
        d = (const char*)st_depth[slot];
        c = (const char*)st_color[slot];
    }
    const bool mask = (flags & TSDF_DEPTH_INVALID_65535) && dk == TSDF_DEPTH_U16_MM;
    if (mask && (dmask_px < npx || !dmask_set[n_sets - 1])) {
        TSDF_TRY(sync_all());
        for (int k = 0; k < kSets; ++k) {
            if (dmask_set[k]) TSDF_HIP(hipFree(dmask_set[k]));
            dmask_set[k] = nullptr;
        }
        for (int k = 0; k < n_sets; ++k)
            TSDF_HIP(hipMalloc(&dmask_set[k], sizeof(unsigned short) * npx * batch));
        dmask_px = npx;
    }
    use_set(cur_set);  // (re)read the set's pointers: the buffers above may be new
    bt->n = n;
    const bool tex = texel_now && dk == TSDF_DEPTH_U16_MM && ck == TSDF_COLOR_RGB8;
    bt->texel = tex ? 1 : 0;
    for (int i = 0; i < n; ++i) {
        Frame* fr = &bt->f[i];
        const double* T = Tinv + 16 * (size_t)(first + i);
        for (int r = 0; r < 12; ++r) fr->T[r] = T[r];
        fr->fx = (double)(float)K[0];
        fr->fy = (double)(float)K[4];
        fr->cx = (double)(float)K[2];
        fr->cy = (double)(float)K[5];
        const double margin = frame_margin(W, H, fr->cx, fr->cy);
        fr->half_m = 0.5 - margin;
        for (int j = 0; j < 4; ++j) {
            fr->Tf[j] = T[j] * fr->fx;
            fr->Tf[4 + j] = T[4 + j] * fr->fy;
        }
        {  // the fast path's depth limit (fold_bound) as the high dword of a positive f64, rounded up
            double wmax[3];
            for (int a = 0; a < 3; ++a) {
                const long long gmax = (a == 0 ? (long long)vol.off[0] + col_gx(vol, vol.nb[0] - 1) + kBrickEdge
                                               : (long long)vol.off[a] + vol.dims[a]);
                wmax[a] = fabs((double)vol.origin[a]) + vol.vs * (double)gmax + 1.0;
            }
            const double zmin = fold_bound(T, fr->fx, fr->fy, wmax, margin);
            long long bits;
            std::memcpy(&bits, &zmin, sizeof bits);
            const long long hi = (std::isfinite(zmin) && zmin < 1e300) ? (bits >> 32) + 1 : 0x7FEFFFFFll;
            fr->zmin_hi = (int)std::min<long long>(hi, 0x7FEFFFFFll);
        }
        fr->ow = ow ? ow[first + i] : ow_default;
        fr->ow32 = (float)fr->ow;
        fr->H = H;
        fr->W = W;
        fr->depth_src = d + dbytes * i;
        fr->depth_mask = mask ? dmask + npx * i : nullptr;
        fr->depth = mask ? (const void*)fr->depth_mask : fr->depth_src;
        fr->color = c + cbytes * i;
        // in place where the byte after the frame is readable: a staging slot (padded, stage_alloc)
        // or a device array with more of the call's frames after this one; else the RGBX copy
        const bool direct = ck == TSDF_COLOR_RGB8 && rgb_direct &&
                            (!(flags & TSDF_DEVICE_PTRS) || (call_color_end && (const char*)fr->color + cbytes < call_color_end));
        if (tex) fr->rgbx = rgbx + 2 * npx * i;  // the prep's 8-byte texels
        else fr->rgbx = direct ? nullptr : rgbx + npx * i;
        fr->pyr = pyr + (size_t)lay.total * i;

        frustum_planes(fr, T, W, H);
    }
    for (int L = 0; L <= kPyrLevels; ++L) {
        bt->pg.off[L] = lay.off[L];
        bt->pg.w[L] = lay.w[L];
        bt->pg.h[L] = lay.h[L];
    }
    return TSDF_OK;
}

int Base::stage_alloc(size_t dbytes, size_t cbytes) {
    if (st_depth_bytes >= dbytes * batch && st_color_bytes >= cbytes * batch) return TSDF_OK;
    TSDF_TRY(sync_all());
    for (int k = 0; k < kSlots; ++k) {
        if (st_depth[k]) TSDF_HIP(hipFree(st_depth[k]));
        if (st_color[k]) TSDF_HIP(hipFree(st_color[k]));
        if (hst_depth[k]) TSDF_HIP(hipHostFree(hst_depth[k]));
        if (hst_color[k]) TSDF_HIP(hipHostFree(hst_color[k]));
        st_depth[k] = st_color[k] = hst_depth[k] = hst_color[k] = nullptr;
    }
    st_depth_bytes = st_color_bytes = 0;
    for (int k = 0; k < kSlots; ++k) {
        TSDF_HIP(hipMalloc(&st_depth[k], dbytes * batch));
        TSDF_HIP(hipMalloc(&st_color[k], cbytes * batch + 64));  // (+ the byte frame_bufs may read past the last frame)
        TSDF_HIP(hipHostMalloc(&hst_depth[k], dbytes * batch, hipHostMallocDefault));
        TSDF_HIP(hipHostMalloc(&hst_color[k], cbytes * batch, hipHostMallocDefault));
    }
    st_depth_bytes = dbytes * batch;
    st_color_bytes = cbytes * batch;
    return TSDF_OK;
}

bool Base::defer_same(int dk, int ck, int H, int W, const double* K) const {
    return dfr.dk_in == dk && dfr.ck == ck && dfr.H == H && dfr.W == W && std::memcmp(dfr.K, K, sizeof(dfr.K)) == 0;
}

int Base::defer_push(const void* depth, int dk, const void* color, int ck, int H, int W,
                     const double* K, const double* T, double ow) {
    const size_t cbytes = frame_bytes_color(ck, H, W), npx = (size_t)H * W;
    if (dfr.n == 0) {
        TSDF_TRY(stage_alloc(frame_bytes_depth(dk, H, W), cbytes));  // (sized for the caller's kind)
        dfr.slot = defer_next;
        dfr.copied = 0;
        defer_next = (defer_next + 1) % kSlots;
        TSDF_HIP(hipEventSynchronize(ev_copied[dfr.slot]));  // its previous DMA has finished
        dfr.dk_in = dk;
        dfr.dk = dk;
        dfr.ck = ck;
        dfr.H = H;
        dfr.W = W;
        std::memcpy(dfr.K, K, sizeof(dfr.K));
    }
    const int i = dfr.n;
    // f64 metres that are all RN(k / 1000) -- the demos' png / 1000. -- go as u16 millimetres: a
    // quarter of the bytes into the bounce slot and over PCIe, the same metres in the kernels
    // (depth_mm_any); a batch holds one kind, so a frame that does not convert after u16 ones
    // sends the caller back to flush them first (kDeferFlush), and then starts an f64 batch
    // (after such a frame the next kMmBackoff batches go as f64 without trying: mm_backoff).  The
    // depth and the colour go through the copy pool as one job.
    const bool try_mm = i == 0 ? mm_backoff == 0 : dfr.dk == TSDF_DEPTH_U16_MM;
    if (i == 0 && mm_backoff > 0) --mm_backoff;
    char* const cdst = (char*)hst_color[dfr.slot] + cbytes * i;
    if (dk == TSDF_DEPTH_F64_M && defer_mm && try_mm) {
        if (CopyPool::get().frame(true, (unsigned short*)hst_depth[dfr.slot] + npx * i, depth, npx, cdst, color,
                                  cbytes)) {
            dfr.dk = TSDF_DEPTH_U16_MM;
        } else {
            mm_backoff = kMmBackoff;
            if (i > 0) return kDeferFlush;
            dfr.dk = TSDF_DEPTH_F64_M;  // (the colour is in place: copy the depth as it is)
            CopyPool::get().copy(hst_depth[dfr.slot], depth, frame_bytes_depth(dfr.dk, H, W));
        }
    } else {
        const size_t db = frame_bytes_depth(dfr.dk, H, W);
        CopyPool::get().frame(false, (char*)hst_depth[dfr.slot] + db * i, depth, db, cdst, color, cbytes);
    }
    const size_t dbytes = frame_bytes_depth(dfr.dk, H, W);
    std::memcpy(dfr.T + 16 * i, T, 16 * sizeof(double));
    dfr.ow[i] = ow;
    dfr.n = i + 1;
    if (dfr.n - dfr.copied >= dma_grain && dfr.n < defer_frames) {
        // the batch's DMA runs as its frames arrive, dma_grain frames at a time (one transfer per
        // field), so that at the flush at most dma_grain frames are still to cross PCIe before the
        // batch's launches can run: the hash flush waits for the previous batch's pool report, i.e.
        // for that batch's DMA and launches, which with one DMA per batch took longer than the
        // host's copies of the next 8 frames (tools/gpu/dropin_trace.py, profiles/r05_dropin/)
        if (dfr.copied == 0) TSDF_HIP(hipStreamWaitEvent(cstream, ev_free[dfr.slot], 0));
        const size_t c0 = (size_t)dfr.copied, nc = (size_t)(dfr.n - dfr.copied);
        TSDF_HIP(hipMemcpyAsync((char*)st_depth[dfr.slot] + dbytes * c0, (const char*)hst_depth[dfr.slot] + dbytes * c0,
                                dbytes * nc, hipMemcpyHostToDevice, cstream));
        TSDF_HIP(hipMemcpyAsync((char*)st_color[dfr.slot] + cbytes * c0, (const char*)hst_color[dfr.slot] + cbytes * c0,
                                cbytes * nc, hipMemcpyHostToDevice, cstream));
        dfr.copied = dfr.n;
    }
    return TSDF_OK;
}

int Base::begin_call(const void* depth, size_t dbytes, const void* color, size_t cbytes, int flags) {
    (void)depth, (void)dbytes;
    call_color_end = (flags & TSDF_DEVICE_PTRS) ? (const char*)color + cbytes : nullptr;
    return TSDF_OK;
}

int Base::end_batch(int flags, int slot) {
    if (prestaged >= 0) slot = prestaged;
    if (!(flags & TSDF_DEVICE_PTRS)) TSDF_HIP(hipEventRecord(ev_free[slot], stream));
    return TSDF_OK;
}

int Base::end_call(int flags) {
    (void)flags;  // the host arrays were fully read into the bounce slots before this point
    call_color_end = nullptr;
    return TSDF_OK;
}

int Base::launch_prep(const Batch& bt, int dk, int ck, int W, int H, hipStream_t stream) {
    dim3 grid((W + 63) / 64, (H + 63) / 64, bt.n);
    bool vec = ck == TSDF_COLOR_RGB8 && W % 4 == 0;
    const unsigned dal = dk == TSDF_DEPTH_U16_MM ? 8u : 16u;
    for (int i = 0; i < bt.n && vec; ++i)  // 8/16-byte depth, 4-byte colour, 16-byte RGBX rows
        vec = ((uintptr_t)bt.f[i].depth_src % dal == 0) && ((uintptr_t)bt.f[i].color % 4 == 0) &&
              ((uintptr_t)bt.f[i].rgbx % 16 == 0) && ((uintptr_t)bt.f[i].depth_mask % 8 == 0);
    if (vec && dk == TSDF_DEPTH_U16_MM)
        hipLaunchKernelGGL(k_prep_vec<0>, grid, dim3(512), 0, stream, bt, count);
    else if (vec)
        hipLaunchKernelGGL(k_prep_vec<1>, grid, dim3(512), 0, stream, bt, count);
    else if (dk == TSDF_DEPTH_U16_MM && ck == TSDF_COLOR_RGB8)
        hipLaunchKernelGGL((k_prep<0, 0>), grid, dim3(1024), 0, stream, bt, count);
    else if (dk == TSDF_DEPTH_U16_MM)
        hipLaunchKernelGGL((k_prep<0, 1>), grid, dim3(1024), 0, stream, bt, count);
    else if (ck == TSDF_COLOR_RGB8)
        hipLaunchKernelGGL((k_prep<1, 0>), grid, dim3(1024), 0, stream, bt, count);
    else
        hipLaunchKernelGGL((k_prep<1, 1>), grid, dim3(1024), 0, stream, bt, count);
    TSDF_HIP(hipGetLastError());
    return TSDF_OK;
}

unsigned Base::grid_for(const void* kernel, int wg) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, wg, 0) != hipSuccess || per_cu < 1)
        per_cu = 1024 / wg;
    long long g = (long long)per_cu * n_cu;
    const long long need = (n_bricks + (wg / 64) - 1) / (wg / 64);
    if (g > need) g = need;
    return (unsigned)(g < 1 ? 1 : g);
}

int Base::check_canon(long long n_vox) {
    int* d = nullptr;
    int bad = 0;
    TSDF_HIP(hipMalloc(&d, sizeof(int)));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(int), stream);
    if (e == hipSuccess && n_vox > 0) {
        const long long want = (n_vox + 255) / 256;
        hipLaunchKernelGGL(k_check_canon, dim3((unsigned)std::min<long long>(want, (long long)n_cu * 16)), dim3(256),
                           0, stream, pool.weight, pool.color, (size_t)n_vox, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, d, sizeof(int), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(d);
    TSDF_HIP(e);
    vol.canon = bad ? 0 : 1;
    return TSDF_OK;
}

int Base::read_stats(tsdf_stats_t* out, int reset) {
    if (!out) return set_error(TSDF_E_ARG, "null stats pointer");
    std::vector<unsigned long long> h(kNStat * kStatSpread);
    TSDF_HIP(hipMemcpyAsync(h.data(), stats, sizeof(unsigned long long) * h.size(),
                            hipMemcpyDeviceToHost, stream));
    TSDF_HIP(hipStreamSynchronize(stream));
    TSDF_TRY(prof.collect());
    unsigned long long s[kNStat] = {0};
    for (int k = 0; k < kNStat; ++k)
        for (int j = 0; j < kStatSpread; ++j) {
            const unsigned long long x = h[k * kStatSpread + j];
            if (k == ST_PROBE_MAX) s[k] = x > s[k] ? x : s[k];
            else s[k] += x;
        }
    std::memset(out, 0, sizeof(*out));
    out->frames = frames;
    out->voxel_updates = (int64_t)s[ST_VOXELS];
    out->bricks_visited = (int64_t)s[ST_VISITED];
    out->bricks_touched = (int64_t)s[ST_TOUCHED];
    out->blocks_allocated = (int64_t)s[ST_ALLOC];
    out->probe_steps = (int64_t)s[ST_PROBE];
    out->probe_max = (int64_t)s[ST_PROBE_MAX];
    out->lookups = (int64_t)s[ST_LOOKUPS];
    out->kernel_ms = prof.ms;
    out->kernel_launches = prof.launches;
    out->bricks_skipped = (int64_t)s[ST_OVERFLOW];
    out->list_errors = (int64_t)s[ST_BAD_ENTRY];
    out->batch_voxels = (int64_t)s[ST_UNIQUE];
    if (reset) {
        TSDF_HIP(hipMemsetAsync(stats, 0, sizeof(unsigned long long) * h.size(), stream));
        TSDF_HIP(hipStreamSynchronize(stream));
        frames = 0;
        prof.ms = 0.0;
        prof.launches = 0;
    }
    return TSDF_OK;
}

int Base::set_profiling(int on) {
    TSDF_TRY(prof.collect());
    prof.on = on != 0;
    return TSDF_OK;
}

void Base::release() {
    if (stream) (void)hipStreamSynchronize(stream);
    prof.release();
    for (int k = 0; k < kSets; ++k) {
        if (pyr_set[k]) (void)hipFree(pyr_set[k]);
        if (rgbx_set[k]) (void)hipFree(rgbx_set[k]);
        if (list_set[k]) (void)hipFree(list_set[k]);
        if (count_set[k]) (void)hipFree(count_set[k]);
        if (dmask_set[k]) (void)hipFree(dmask_set[k]);
        pyr_set[k] = nullptr;
        rgbx_set[k] = nullptr;
        list_set[k] = nullptr;
        count_set[k] = nullptr;
        dmask_set[k] = nullptr;
    }
    n_sets = 1;
    if (rcp) (void)hipFree(rcp);
    rcp = nullptr;
    if (stats) (void)hipFree(stats);
    if (cstream) (void)hipStreamSynchronize(cstream);
    for (int k = 0; k < kSlots; ++k) {
        if (st_depth[k]) (void)hipFree(st_depth[k]);
        if (st_color[k]) (void)hipFree(st_color[k]);
        if (ev_copied[k]) (void)hipEventDestroy(ev_copied[k]);
        if (ev_free[k]) (void)hipEventDestroy(ev_free[k]);
        st_depth[k] = st_color[k] = nullptr;
        ev_copied[k] = ev_free[k] = nullptr;
    }
    dmask = nullptr;
    for (int k = 0; k < kSlots; ++k) {
        if (hst_depth[k]) (void)hipHostFree(hst_depth[k]);
        if (hst_color[k]) (void)hipHostFree(hst_color[k]);
        hst_depth[k] = hst_color[k] = nullptr;
    }
    if (cstream) (void)hipStreamDestroy(cstream);
    cstream = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    pyr = nullptr;
    rgbx = nullptr;
    list = nullptr;
    count = nullptr;
    stats = nullptr;
    stream = nullptr;
}

__global__ void k_hash_keys(const long long* xyz, long long n, long long m, int bits, long long* out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ref_hash(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], m, bits);
}

}  // namespace tsdf

using namespace tsdf;

extern "C" {

const char* tsdf_last_error(void) { return g_err.c_str(); }

int tsdf_device_count(int* n) {
    if (!n) return set_error(TSDF_E_ARG, "null pointer");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return TSDF_OK;
}

int tsdf_hash_keys(const int64_t* xyz, int64_t n, int64_t table_size, int int_bits, int64_t* out,
                   int device) {
    if (n < 0 || (n > 0 && (!xyz || !out)) || table_size <= 0 || (int_bits != 32 && int_bits != 64))
        return set_error(TSDF_E_ARG, "tsdf_hash_keys: bad arguments");
    if (n == 0) return TSDF_OK;
    TSDF_HIP(hipSetDevice(device));
    long long *dx = nullptr, *dout = nullptr;
    TSDF_HIP(hipMalloc(&dx, sizeof(long long) * 3 * n));
    TSDF_HIP(hipMalloc(&dout, sizeof(long long) * n));
    TSDF_HIP(hipMemcpy(dx, xyz, sizeof(long long) * 3 * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_hash_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr,
                       (const long long*)dx, (long long)n, (long long)table_size, int_bits, dout);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(long long) * n, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dout);
    TSDF_HIP(e);
    return TSDF_OK;
}

}  // extern "C"
