// tsdf_dense.hip -- dense TSDF grid: the MI355X replacement of TSDFVolume
// (grid_fusion.py:19-320).  HBM layout: three f32 SoA arrays of 512-voxel bricks, brick b =
// (bx*nby + by)*nbz + bz, brick-local voxel (x*8 + y)*8 + z.
#include <algorithm>
#include <vector>
#include <cstdlib>
#include <cstring>

#include "tsdf_host.h"

using namespace tsdf;

struct tsdf_dense {
    Base b;
    Mesh mesh;
    int nz = 4;  // z-steps per wave in k_integrate (8: a brick per wave; 4: a z-half per wave)
    bool fused = true;  // three-stage pipeline launches (k_fused) when a call allows them
    int gi_per_cu = 0;  // integrate workgroups per CU in a fused launch (0: as many as fit)
};

namespace {

__global__ void k_fill3(float* t, float* w, float* c, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        t[i] = 1.0f;
        w[i] = 0.0f;
        c[i] = 0.0f;
    }
}

// brick layout <-> C-order rows of the shard: C-order row i of the buffer is local x row
// rows[i] (rows == nullptr: row0 + i).  TO_CORDER: buffer <- bricks, else bricks <- buffer.
template <bool TO_CORDER>
__global__ void k_rows(Vol v, const long long* __restrict__ rows, long long row0, long long nrows,
                       float* __restrict__ bricks, float* __restrict__ buf) {
    const size_t yz = (size_t)v.dims[1] * v.dims[2];
    const size_t n = (size_t)nrows * yz;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int z = (int)(i % v.dims[2]);
        const size_t ry = i / v.dims[2];
        const int y = (int)(ry % v.dims[1]);
        const long long r = (long long)(ry / v.dims[1]);
        const int x = (int)(rows ? rows[r] : row0 + r);
        const size_t b = ((size_t)(x >> 3) * v.nb[1] + (y >> 3)) * v.nb[2] + (z >> 3);
        const size_t j = b * kBrickVox + (size_t)((x & 7) * 8 + (y & 7)) * 8 + (z & 7);
        if (TO_CORDER) buf[i] = bricks[j];
        else bricks[j] = buf[i];
    }
}

// The in-line path: per batch prep, cull and integrate, one after the other on the handle's
// stream.  Serves every input format.
int dense_run_inline(tsdf_dense* h, int n_frames, const void* depth, int dk, const void* color, int ck,
                     int H, int W, const double* K, const double* Tinv, const double* ow, int flags) {
    Base& B = h->b;
    const Table no_table{};
    const unsigned cull_grid = B.cull_grid();
    const unsigned grid = h->nz == 4 ? 2 * B.grid_for((const void*)k_integrate<false, 0, 0, true, 4>)
                                     : B.grid_for((const void*)k_integrate<false, 0, 0, true, 8>);
    B.use_set(0);
    const int nbat = B.batch;
    for (int f0 = 0; f0 < n_frames; f0 += nbat) {
        Batch bt;
        const int n = n_frames - f0 < nbat ? n_frames - f0 : nbat;
        const int slot = (f0 / nbat) % kSlots;
        TSDF_TRY(B.prepare_batch(&bt, depth, dk, color, ck, H, W, K, Tinv, ow, 1.0, flags, f0, n, slot));
        TSDF_TRY(B.launch_prep(bt, dk, ck, W, H, B.stream));
        hipLaunchKernelGGL((k_cull<false>), dim3(cull_grid), dim3(kCullWG), 0, B.stream, B.vol, bt, no_table,
                           B.list, B.count, B.stats);
        TSDF_HIP(hipGetLastError());
        hipEvent_t e0;
        TSDF_TRY(B.prof.begin(B.stream, &e0));
        bool ow1 = true;
        for (int i = 0; i < n; ++i) ow1 = ow1 && bt.f[i].ow == 1.0;
        const ListEntry* L = B.list;
        const int sel = (dk == TSDF_DEPTH_U16_MM ? 0 : 4) | (ck == TSDF_COLOR_RGB8 ? 0 : 2) | (ow1 ? 1 : 0) |
                        (h->nz == 4 ? 8 : 0);
        switch (sel) {
#define TSDF_LAUNCH(S, DK_, CK_, OW_, NZ_)                                                             \
    case S:                                                                                            \
        hipLaunchKernelGGL((k_integrate<false, DK_, CK_, OW_, NZ_>), dim3(grid), dim3(kWG), 0, B.stream,   \
                           B.vol, bt, B.pool, no_table, B.stats, L, B.count, 0);                       \
        break;
            TSDF_LAUNCH(0, 0, 0, false, 8)
            TSDF_LAUNCH(1, 0, 0, true, 8)
            TSDF_LAUNCH(2, 0, 1, false, 8)
            TSDF_LAUNCH(3, 0, 1, true, 8)
            TSDF_LAUNCH(4, 1, 0, false, 8)
            TSDF_LAUNCH(5, 1, 0, true, 8)
            TSDF_LAUNCH(6, 1, 1, false, 8)
            TSDF_LAUNCH(7, 1, 1, true, 8)
            TSDF_LAUNCH(8, 0, 0, false, 4)
            TSDF_LAUNCH(9, 0, 0, true, 4)
            TSDF_LAUNCH(10, 0, 1, false, 4)
            TSDF_LAUNCH(11, 0, 1, true, 4)
            TSDF_LAUNCH(12, 1, 0, false, 4)
            TSDF_LAUNCH(13, 1, 0, true, 4)
            TSDF_LAUNCH(14, 1, 1, false, 4)
            TSDF_LAUNCH(15, 1, 1, true, 4)
#undef TSDF_LAUNCH
        }
        TSDF_HIP(hipGetLastError());
        TSDF_TRY(B.prof.end(B.stream, e0));
        TSDF_TRY(B.end_batch(flags, slot));
        B.frames += n;
    }
    return TSDF_OK;
}

// The fused path (k_fused, tsdf_device.h): launch L runs integrate(L), cull(L+1) and prep(L+2)
// of the call's batches, L = -2 .. nb-1.  Batch j uses buffer set and staging slot j % kSets.
// u16 depth + RGB8 with the vectorised prep's alignment only (the bench's and the demos' case).
int dense_run_fused(tsdf_dense* h, int n_frames, const void* depth, int dk, const void* color, int H,
                    int W, const double* K, const double* Tinv, const double* ow, int flags) {
    Base& B = h->b;
    TSDF_TRY(B.use_sets(kSets));
    const int nbat = B.batch;
    const int nb = (n_frames + nbat - 1) / nbat;
    const int gi_occ = h->nz == 4 ? (int)B.grid_for((const void*)k_fused<true, 4>, kFusedWG)
                                  : (int)B.grid_for((const void*)k_fused<true, 8>, kFusedWG);
    const int gi_full = h->gi_per_cu ? std::min(gi_occ, h->gi_per_cu * B.n_cu) : gi_occ;
    const int gc_full = (int)B.cull_grid_fused();
    // texels (Base::texel_for; z-half waves only) for the batches this call prepares
    const bool tex = h->nz == 4 && B.texel_for(dk, B.n_bricks, Base::kTexelMinBricksDense);
    struct TexelScope {
        Base& b;
        ~TexelScope() { b.texel_now = false; }
    } tex_scope{B};
    B.texel_now = tex;
    Batch bts[kSets];
    for (int L = -2; L < nb; ++L) {
        const int jp = L + 2;  // batch prepped by this launch
        if (jp < nb) {
            const int f0 = jp * nbat;
            const int n = n_frames - f0 < nbat ? n_frames - f0 : nbat;
            B.use_set(jp % kSets);
            TSDF_TRY(B.prepare_batch(&bts[jp % kSets], depth, dk, color, TSDF_COLOR_RGB8, H, W,
                                     K, Tinv, ow, 1.0, flags, f0, n, jp % kSlots));
        }
        const bool has_i = L >= 0, has_c = L + 1 >= 0 && L + 1 < nb, has_p = jp < nb;
        static const Batch kNone{};
        const Batch& bi = has_i ? bts[L % kSets] : kNone;
        const Batch& bc = has_c ? bts[(L + 1) % kSets] : kNone;
        const Batch& bp = has_p ? bts[jp % kSets] : kNone;
        Stage sg{};
        sg.gi = has_i ? gi_full : 0;
        sg.gc = has_c ? gc_full : 0;
        sg.cg = B.cull_per_wg();
        sg.ptx = (W + 63) / 64;
        sg.pty = (H + 63) / 64;
        if (has_i) {
            sg.list_i = B.list_set[L % kSets];
            sg.count_i = B.count_set[L % kSets];
        }
        if (has_c) {
            sg.list_c = B.list_set[(L + 1) % kSets];
            sg.count_c = B.count_set[(L + 1) % kSets];
        }
        if (has_p) sg.count_p = B.count_set[jp % kSets];
        const long long grid = (long long)sg.gi + sg.gc + (has_p ? (long long)sg.ptx * sg.pty * bp.n : 0);
        if (grid >= (1ll << 31)) return set_error(TSDF_E_ARG, "fused grid too large");
        bool ow1 = true;
        for (int i = 0; i < bi.n; ++i) ow1 = ow1 && bi.f[i].ow == 1.0;
        hipEvent_t e0 = nullptr;
        if (has_i) TSDF_TRY(B.prof.begin(B.stream, &e0));
        // (u32 colour registers where the volume is canonical: obs_weight 1 and NZ = 4, tsdf_device.h)
        const bool cu = TSDF_COLOR_U32 && ow1 && h->nz == 4 && B.vol.canon;
        const int sel = (ow1 ? 1 : 0) | (h->nz == 4 ? 2 : 0) | (dk == TSDF_DEPTH_U16_MM ? 0 : 4) | (cu ? 8 : 0) |
                        (tex ? 16 : 0);
        const FusedArgs args{B.vol, bi, bc, bp, B.pool, B.stats, sg};
        switch (sel) {
#define TSDF_LAUNCH(S, OW_, NZ_, DK_)                                                                   \
    case S:                                                                                             \
        hipLaunchKernelGGL((k_fused<OW_, NZ_, DK_>), dim3((unsigned)grid), dim3(kFusedWG), 0, B.stream, args); \
        break;
#define TSDF_LAUNCH_CU(S, OW_, NZ_, DK_)                                                                \
    case S:                                                                                             \
        hipLaunchKernelGGL((k_fused<OW_, NZ_, DK_, true>), dim3((unsigned)grid), dim3(kFusedWG), 0, B.stream, args); \
        break;
            TSDF_LAUNCH(0, false, 8, 0)
            TSDF_LAUNCH(1, true, 8, 0)
            TSDF_LAUNCH(2, false, 4, 0)
            TSDF_LAUNCH(3, true, 4, 0)
            TSDF_LAUNCH(4, false, 8, 1)
            TSDF_LAUNCH(5, true, 8, 1)
            TSDF_LAUNCH(6, false, 4, 1)
            TSDF_LAUNCH(7, true, 4, 1)
            TSDF_LAUNCH_CU(11, true, 4, 0)
            TSDF_LAUNCH_CU(15, true, 4, 1)
            TSDF_LAUNCH(18, false, 4, 2)
            TSDF_LAUNCH(19, true, 4, 2)
            TSDF_LAUNCH_CU(27, true, 4, 2)
#undef TSDF_LAUNCH
#undef TSDF_LAUNCH_CU
        }
        TSDF_HIP(hipGetLastError());
        if (has_i) {
            TSDF_TRY(B.prof.end(B.stream, e0));
            TSDF_TRY(B.end_batch(flags, L % kSlots));  // batch L's frames: last read by this launch
            B.frames += bi.n;
        }
    }
    return TSDF_OK;
}

int dense_run(tsdf_dense* h, int n_frames, const void* depth, int dk, const void* color, int ck,
              int H, int W, const double* K, const double* Tinv, const double* ow, int flags) {
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(B.begin_call(depth, frame_bytes_depth(dk, H, W) * n_frames, color,
                          frame_bytes_color(ck, H, W) * n_frames, flags));
    CallGuard guard(B, flags);
    B.note_frames(ck, ow, n_frames, 1.0);
    // the fused pipeline needs the vectorised prep: u16 or f64 depth + RGB8, W % 4 == 0 and
    // (device frames) 8-byte u16 / 16-byte f64 depth and 4-byte colour alignment of every frame
    // (host frames are staged aligned)
    bool fused = h->fused && ck == TSDF_COLOR_RGB8 && W % 4 == 0 && n_frames > 0;
    if (fused && (flags & TSDF_DEVICE_PTRS))
        fused = (uintptr_t)depth % (dk == TSDF_DEPTH_U16_MM ? 8 : 16) == 0 && (uintptr_t)color % 4 == 0 &&
                ((size_t)H * W) % 4 == 0;
    if (fused) TSDF_TRY(dense_run_fused(h, n_frames, depth, dk, color, H, W, K, Tinv, ow, flags));
    else TSDF_TRY(dense_run_inline(h, n_frames, depth, dk, color, ck, H, W, K, Tinv, ow, flags));
    TSDF_TRY(guard.finish());
    if (!(flags & TSDF_ASYNC)) TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

// Run the deferred frames (TSDF_DEFER) as one asynchronous batch from their bounce slot.
int dense_flush(tsdf_dense* h) {
    Base& B = h->b;
    if (B.dfr.n == 0) return TSDF_OK;
    const Base::Deferred d = B.dfr;
    B.dfr.n = 0;
    B.prestaged = d.slot;
    B.pre_copied = d.copied;
    const int r = dense_run(h, d.n, B.hst_depth[d.slot], d.dk, B.hst_color[d.slot], d.ck, d.H, d.W, d.K, d.T,
                            d.ow, TSDF_ASYNC);
    B.prestaged = -1;
    B.pre_copied = 0;
    return r;
}

// C-order get/set of the whole shard through a bounded device buffer (<= 64 MiB of rows at a time).
int dense_xfer(tsdf_dense* h, float* tsdf_, float* weight_, float* color_, bool get) {
    Base& B = h->b;
    TSDF_TRY(dense_flush(h));
    TSDF_HIP(hipSetDevice(B.device));
    const size_t yz = (size_t)B.vol.dims[1] * B.vol.dims[2];
    const long long X = B.vol.dims[0];
    const long long chunk = std::max<long long>(1, std::min<long long>(X, (64ll << 20) / (long long)(yz * sizeof(float))));
    float* tmp = nullptr;
    TSDF_HIP(hipMalloc(&tmp, (size_t)chunk * yz * sizeof(float)));
    float* host[3] = {tsdf_, weight_, color_};
    float* dev[3] = {B.pool.tsdf, B.pool.weight, B.pool.color};
    hipError_t e = hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>(((size_t)chunk * yz + 255) / 256, (size_t)B.n_cu * 16);
    for (int k = 0; k < 3 && e == hipSuccess; ++k) {
        if (!host[k]) continue;
        for (long long r0 = 0; r0 < X && e == hipSuccess; r0 += chunk) {
            const long long nr = std::min(chunk, X - r0);
            const size_t bytes = (size_t)nr * yz * sizeof(float);
            if (get) {
                hipLaunchKernelGGL(k_rows<true>, dim3(grid), dim3(256), 0, B.stream, B.vol, (const long long*)nullptr, r0,
                                   nr, dev[k], tmp);
                e = hipGetLastError();
                if (e == hipSuccess) e = hipMemcpyAsync(host[k] + (size_t)r0 * yz, tmp, bytes, hipMemcpyDeviceToHost, B.stream);
            } else {
                e = hipMemcpyAsync(tmp, host[k] + (size_t)r0 * yz, bytes, hipMemcpyHostToDevice, B.stream);
                if (e == hipSuccess) {
                    hipLaunchKernelGGL(k_rows<false>, dim3(grid), dim3(256), 0, B.stream, B.vol, (const long long*)nullptr,
                                       r0, nr, dev[k], tmp);
                    e = hipGetLastError();
                }
            }
            if (e == hipSuccess) e = hipStreamSynchronize(B.stream);  // tmp is reused by the next chunk
        }
    }
    (void)hipFree(tmp);
    TSDF_HIP(e);
    return TSDF_OK;
}

struct DevPtrs {
    std::vector<void*> p;
    ~DevPtrs() {
        for (void* q : p)
            if (q) (void)hipFree(q);
    }
};

}  // namespace

Base* tsdf::dense_base(tsdf_dense_t* d) { return &d->b; }

extern "C" {

static int dense_create(const int64_t dims[3], const int64_t index_offset[3], int xstride, int xodd,
                        const float origin[3], double voxel_size, double trunc, int device,
                        tsdf_dense_t** out) {
    *out = nullptr;
    tsdf_dense* h = new tsdf_dense();
    int r = h->b.init(device, dims, index_offset, origin, voxel_size, trunc);
    if (r == TSDF_OK) {
        h->b.vol.xstride = xstride;
        h->b.vol.xodd = xodd;
        if (const char* e = getenv("TSDF_DENSE_NZ")) h->nz = atoi(e) == 8 ? 8 : 4;  // A/B override
        if (xstride > kBrickEdge) {  // cyclic shard: superbricks one column wide, 8x8 in y, z
            h->b.vol.sb[0] = 0;
            h->b.vol.sb[1] = h->b.vol.sb[2] = 3;
        }
        r = h->b.set_batch(xstride > kBrickEdge ? kMaxBatch : kFullBatch);
        const int64_t last = h->b.vol.nb[0] - 1;
        const int64_t gx_max = (int64_t)h->b.vol.off[0] + (last >> 1) * 2 * (int64_t)xstride + (last & 1) * (int64_t)xodd + kBrickEdge;
        if (r == TSDF_OK && gx_max > (1 << 24)) r = set_error(TSDF_E_ARG, "shard x extent out of range");
    }
    if (r == TSDF_OK) {
        // three-stage pipeline launches; TSDF_PIPELINE=0 forces the in-line path
        if (const char* e = getenv("TSDF_PIPELINE")) h->fused = atoi(e) != 0;
        if (const char* e = getenv("TSDF_FUSED_GI_PER_CU")) h->gi_per_cu = std::max(0, atoi(e));  // A/B override
    }
    if (r == TSDF_OK) {
        const size_t n = (size_t)h->b.n_bricks * kBrickVox * sizeof(float);
        hipError_t e = hipMalloc(&h->b.pool.tsdf, n);
        if (e == hipSuccess) e = hipMalloc(&h->b.pool.weight, n);
        if (e == hipSuccess) e = hipMalloc(&h->b.pool.color, n);
        if (e != hipSuccess)
            r = set_error(e == hipErrorOutOfMemory ? TSDF_E_OOM : TSDF_E_HIP,
                          "allocating %zu bytes of brick state: %s", 3 * n, hipGetErrorString(e));
    }
    if (r == TSDF_OK) r = tsdf_dense_reset(h);
    if (r != TSDF_OK) {
        std::string keep = tsdf_last_error();
        tsdf_dense_destroy(h);
        set_error(r, "%s", keep.c_str());
        return r;
    }
    *out = h;
    return TSDF_OK;
}

int tsdf_dense_create(const int64_t dims[3], const int64_t index_offset[3], const float origin[3],
                      double voxel_size, double trunc, int device, tsdf_dense_t** out) {
    if (!dims || !origin || !out) return set_error(TSDF_E_ARG, "null pointer");
    return dense_create(dims, index_offset, kBrickEdge, kBrickEdge, origin, voxel_size, trunc, device, out);
}

int tsdf_dense_create_shard(const int64_t global_dims[3], int shard, int n_shards,
                            const float origin[3], double voxel_size, double trunc, int device,
                            tsdf_dense_t** out) {
    if (!global_dims || !origin || !out) return set_error(TSDF_E_ARG, "null pointer");
    *out = nullptr;
    if (n_shards < 1 || shard < 0 || shard >= n_shards)
        return set_error(TSDF_E_ARG, "shard %d of %d", shard, n_shards);
    const int64_t X = global_dims[0];
    const int64_t cols = (X + kBrickEdge - 1) / kBrickEdge;
    if (X <= 0 || shard >= cols) return set_error(TSDF_E_ARG, "shard %d owns no x-column of %lld voxels", shard, (long long)X);
    // Mirrored pairs: in every period of 2n columns shard s owns s and 2n-1-s, so a work density
    // that drifts along x evens out across the ranks (plain c % n == s handed rank 0 the lightest
    // columns of every period: 1.07 max/mean rank time at 8 ranks on the bench ring).
    const int64_t P = 2 * (int64_t)n_shards, lo = shard, hi = P - 1 - shard;
    const int64_t full = cols / P, rem = cols % P;
    const int64_t mine = 2 * full + (lo < rem) + (hi < rem);
    auto col = [&](int64_t j) { return (j >> 1) * P + ((j & 1) ? hi : lo); };
    const int64_t last = col(mine - 1);
    const int64_t last_w = (last == cols - 1) ? X - last * kBrickEdge : kBrickEdge;
    const int64_t dims[3] = {(mine - 1) * kBrickEdge + last_w, global_dims[1], global_dims[2]};
    const int64_t off[3] = {lo * kBrickEdge, 0, 0};
    if (n_shards == 1)
        return dense_create(dims, off, kBrickEdge, kBrickEdge, origin, voxel_size, trunc, device, out);
    return dense_create(dims, off, kBrickEdge * n_shards, (int)((hi - lo) * kBrickEdge), origin, voxel_size,
                        trunc, device, out);
}

int tsdf_dense_destroy(tsdf_dense_t* h) {
    if (!h) return TSDF_OK;
    (void)hipSetDevice(h->b.device);
    h->mesh.release();
    h->b.release();
    if (h->b.pool.tsdf) (void)hipFree(h->b.pool.tsdf);
    if (h->b.pool.weight) (void)hipFree(h->b.pool.weight);
    if (h->b.pool.color) (void)hipFree(h->b.pool.color);
    delete h;
    return TSDF_OK;
}

int tsdf_dense_reset(tsdf_dense_t* h) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    Base& B = h->b;
    B.dfr.n = 0;  // deferred frames are dropped with the state
    TSDF_HIP(hipSetDevice(B.device));
    hipLaunchKernelGGL(k_fill3, dim3(4096), dim3(256), 0, B.stream, B.pool.tsdf, B.pool.weight,
                       B.pool.color, (size_t)B.n_bricks * kBrickVox);
    TSDF_HIP(hipGetLastError());
    TSDF_HIP(hipMemsetAsync(B.stats, 0, sizeof(unsigned long long) * kNStat * kStatSpread, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    B.frames = 0;
    B.vol.canon = 1;
    return TSDF_OK;
}

int tsdf_dense_integrate(tsdf_dense_t* h, const void* depth, int depth_kind, const void* color,
                         int color_kind, int height, int width, const double K[9],
                         const double world_to_cam[16], double obs_weight, int flags) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_TRY(check_frame_args(depth, depth_kind, color, color_kind, height, width, K, world_to_cam));
    TSDF_HIP(hipSetDevice(h->b.device));
    Base& B = h->b;
    if (flags & TSDF_DEFER) {
        if (flags & TSDF_DEVICE_PTRS) return set_error(TSDF_E_ARG, "TSDF_DEFER takes host frames only");
        if (B.dfr.n > 0 && !B.defer_same(depth_kind, color_kind, height, width, K)) TSDF_TRY(dense_flush(h));
        int r = B.defer_push(depth, depth_kind, color, color_kind, height, width, K, world_to_cam, obs_weight);
        if (r == Base::kDeferFlush) {  // the batch's frames went as u16 and this one cannot
            TSDF_TRY(dense_flush(h));
            r = B.defer_push(depth, depth_kind, color, color_kind, height, width, K, world_to_cam, obs_weight);
        }
        TSDF_TRY(r);
        if (B.dfr.n == B.defer_frames) TSDF_TRY(dense_flush(h));
        return TSDF_OK;
    }
    TSDF_TRY(dense_flush(h));
    return dense_run(h, 1, depth, depth_kind, color, color_kind, height, width, K, world_to_cam,
                     &obs_weight, flags);
}

int tsdf_dense_integrate_batch(tsdf_dense_t* h, int n_frames, const void* depth, int depth_kind,
                               const void* color, int color_kind, int height, int width,
                               const double K[9], const double* world_to_cam,
                               const double* obs_weight, int flags) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    if (n_frames < 0) return set_error(TSDF_E_ARG, "n_frames < 0");
    if (n_frames == 0) return TSDF_OK;
    TSDF_TRY(check_frame_args(depth, depth_kind, color, color_kind, height, width, K, world_to_cam));
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(dense_flush(h));
    return dense_run(h, n_frames, depth, depth_kind, color, color_kind, height, width, K,
                     world_to_cam, obs_weight, flags);
}

int tsdf_dense_get(tsdf_dense_t* h, float* tsdf_, float* weight_, float* color_) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    return dense_xfer(h, tsdf_, weight_, color_, true);
}

int tsdf_dense_set(tsdf_dense_t* h, const float* tsdf_, const float* weight_, const float* color_) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_TRY(dense_xfer(h, (float*)tsdf_, (float*)weight_, (float*)color_, false));
    if (weight_ || color_) TSDF_TRY(h->b.check_canon(h->b.n_bricks * kBrickVox));  // Vol::canon
    return TSDF_OK;
}

int tsdf_dense_frames_per_launch(tsdf_dense_t* h, int* n) {
    if (!h || !n) return set_error(TSDF_E_ARG, "null pointer");
    *n = h->b.batch;
    return TSDF_OK;
}

int tsdf_dense_sync(tsdf_dense_t* h) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(dense_flush(h));
    TSDF_HIP(hipStreamSynchronize(h->b.stream));
    return TSDF_OK;
}

int tsdf_dense_stats(tsdf_dense_t* h, tsdf_stats_t* out, int reset) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(dense_flush(h));
    return h->b.read_stats(out, reset);
}

int tsdf_dense_extract_mesh(tsdf_dense_t* h, int64_t* n_verts, int64_t* n_tris) {
    return tsdf_dense_extract_mesh_halo(h, 0, nullptr, 0, nullptr, nullptr, 0, n_verts, n_tris);
}

int tsdf_dense_mesh_halo_rows(tsdf_dense_t* h, int64_t global_x, int64_t* rows, int64_t* n_rows) {
    if (!h || !n_rows) return set_error(TSDF_E_ARG, "null pointer");
    std::vector<long long> v;
    TSDF_TRY(mesh_halo_rows(h->b.vol, global_x, &v));
    if (rows) {
        if (*n_rows < (int64_t)v.size()) return set_error(TSDF_E_ARG, "rows holds %lld, need %zu", (long long)*n_rows, v.size());
        for (size_t i = 0; i < v.size(); ++i) rows[i] = v[i];
    }
    *n_rows = (int64_t)v.size();
    return TSDF_OK;
}

int tsdf_dense_extract_mesh_halo(tsdf_dense_t* h, int64_t global_x, const int64_t* halo_gx, int64_t n_halo,
                                 const float* halo_tsdf, const float* halo_color, int flags, int64_t* n_verts,
                                 int64_t* n_tris) {
    if (!h || !n_verts || !n_tris || n_halo < 0 || (n_halo > 0 && (!halo_gx || !halo_tsdf || !halo_color)))
        return set_error(TSDF_E_ARG, "bad arguments");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(dense_flush(h));
    MeshDomain d;
    TSDF_TRY(mesh_domain(B.vol, global_x, halo_gx, n_halo, &d));
    const size_t hb = (size_t)n_halo * B.vol.dims[1] * B.vol.dims[2] * sizeof(float);
    const float *ht = halo_tsdf, *hc = halo_color;
    float *ut = nullptr, *uc = nullptr;
    int r = TSDF_OK;
    if (n_halo > 0 && !(flags & TSDF_DEVICE_PTRS)) {  // host halo rows: upload them for the call
        hipError_t e = hipMalloc(&ut, hb);
        if (e == hipSuccess) e = hipMalloc(&uc, hb);
        if (e == hipSuccess) e = hipMemcpyAsync(ut, halo_tsdf, hb, hipMemcpyHostToDevice, B.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(uc, halo_color, hb, hipMemcpyHostToDevice, B.stream);
        if (e != hipSuccess) r = set_error(TSDF_E_HIP, "halo upload: %s", hipGetErrorString(e));
        ht = ut;
        hc = uc;
    } else if (n_halo > 0) {
        TSDF_HIP(hipDeviceSynchronize());  // the caller's producer (e.g. a collective) may be on another stream
    }
    if (r == TSDF_OK) r = extract_mesh(B, B.pool, h->mesh, d, ht, hc);
    if (ut) (void)hipFree(ut);
    if (uc) (void)hipFree(uc);
    TSDF_TRY(r);
    *n_verts = h->mesh.n_verts;
    *n_tris = h->mesh.n_tris;
    return TSDF_OK;
}

int tsdf_dense_get_mesh(tsdf_dense_t* h, float* verts, float* normals, uint8_t* colors, int32_t* faces) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    return copy_mesh(h->b, h->mesh, verts, normals, colors, faces);
}

int tsdf_dense_get_mesh_keys(tsdf_dense_t* h, int64_t* keys) {
    if (!h || !keys) return set_error(TSDF_E_ARG, "null pointer");
    TSDF_HIP(hipSetDevice(h->b.device));
    return copy_mesh(h->b, h->mesh, nullptr, nullptr, nullptr, nullptr, keys);
}

int tsdf_dense_get_rows(tsdf_dense_t* h, const int64_t* rows, int64_t n_rows, float* tsdf_, float* weight_,
                        float* color_, int flags) {
    if (!h || n_rows < 0 || (n_rows > 0 && !rows)) return set_error(TSDF_E_ARG, "bad arguments");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(dense_flush(h));
    if (n_rows == 0) return TSDF_OK;
    for (int64_t i = 0; i < n_rows; ++i)
        if (rows[i] < 0 || rows[i] >= B.vol.dims[0])
            return set_error(TSDF_E_ARG, "local row %lld outside [0, %d)", (long long)rows[i], B.vol.dims[0]);
    const size_t yz = (size_t)B.vol.dims[1] * B.vol.dims[2];
    const size_t bytes = (size_t)n_rows * yz * sizeof(float);
    DevPtrs bufs;
    long long* drows = nullptr;
    TSDF_HIP(hipMalloc(&drows, sizeof(long long) * n_rows));
    bufs.p.push_back(drows);
    TSDF_HIP(hipMemcpyAsync(drows, rows, sizeof(long long) * n_rows, hipMemcpyHostToDevice, B.stream));
    float* out[3] = {tsdf_, weight_, color_};
    float* dev[3] = {B.pool.tsdf, B.pool.weight, B.pool.color};
    const unsigned grid = (unsigned)std::min<size_t>(((size_t)n_rows * yz + 255) / 256, (size_t)B.n_cu * 16);
    for (int k = 0; k < 3; ++k) {
        if (!out[k]) continue;
        float* dst = out[k];
        if (!(flags & TSDF_DEVICE_PTRS)) {
            TSDF_HIP(hipMalloc(&dst, bytes));
            bufs.p.push_back(dst);
        }
        hipLaunchKernelGGL(k_rows<true>, dim3(grid), dim3(256), 0, B.stream, B.vol, (const long long*)drows, 0ll,
                           (long long)n_rows, dev[k], dst);
        TSDF_HIP(hipGetLastError());
        if (!(flags & TSDF_DEVICE_PTRS)) TSDF_HIP(hipMemcpyAsync(out[k], dst, bytes, hipMemcpyDeviceToHost, B.stream));
    }
    TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

int tsdf_dense_set_profiling(tsdf_dense_t* h, int on) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(dense_flush(h));
    return h->b.set_profiling(on);
}

}  // extern "C"

#ifdef TSDF_WG_TIMES
// (diagnostic builds) the last fused launch's per-workgroup start / end / role|items:
// out[4 * kWgTimes]
extern "C" int tsdf_diag_wg_times(unsigned long long* out) {
    TSDF_HIP(hipDeviceSynchronize());
    TSDF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_times), sizeof(unsigned long long) * 4 * kWgTimes));
    static const std::vector<unsigned long long> zero(4 * (size_t)kWgTimes, 0ull);  // (read and cleared)
    TSDF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wg_times), zero.data(), sizeof(unsigned long long) * 4 * kWgTimes));
    return TSDF_OK;
}
#endif

#ifdef TSDF_DIAG
// (diagnostic builds) the integrate's path counters (g_ddiag, csrc/tsdf_device.h), read and cleared
extern "C" int tsdf_diag_counts(unsigned long long* out) {
    TSDF_HIP(hipDeviceSynchronize());
    TSDF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(tsdf::g_ddiag), sizeof(unsigned long long) * 8));
    const unsigned long long zero[8] = {};
    TSDF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(tsdf::g_ddiag), zero, sizeof(zero)));
    return TSDF_OK;
}
#endif
