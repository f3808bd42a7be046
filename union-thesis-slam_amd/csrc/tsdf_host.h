// tsdf_host.h -- host-side internals shared by the dense and hash C-ABI implementations.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "tsdf_device.h"
#include "tsdf_hip.h"

namespace tsdf {

int set_error(int code, const char* fmt, ...);

#define TSDF_HIP(expr)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return ::tsdf::set_error(e_ == hipErrorOutOfMemory ? TSDF_E_OOM : TSDF_E_HIP,     \
                                     "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                                     __FILE__, __LINE__);                                     \
    } while (0)

#define TSDF_TRY(expr)            \
    do {                          \
        int r_ = (expr);          \
        if (r_ != TSDF_OK) return r_; \
    } while (0)

inline size_t frame_bytes_depth(int dk, int H, int W) { return (size_t)H * W * (dk == TSDF_DEPTH_U16_MM ? 2 : 8); }
inline size_t frame_bytes_color(int ck, int H, int W) { return (size_t)H * W * (ck == TSDF_COLOR_RGB8 ? 3 : 4); }

struct PyrLayout {
    int off[kPyrLevels + 1];
    int w[kPyrLevels + 1];
    int h[kPyrLevels + 1];
    int total;
};
PyrLayout pyr_layout(int H, int W);

// HIP-event timing of the integrate kernels (tsdf_*_set_profiling).
struct Profiler {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<hipEvent_t> spare;
    double ms = 0.0;
    long long launches = 0;
    int begin(hipStream_t s, hipEvent_t* e0);
    int end(hipStream_t s, hipEvent_t e0);
    int collect();  // synchronises on the recorded events and accumulates their spans
    void release();
};

// Buffer sets: batch j of a call uses set j % kSets (the fused dense pipeline has batches k,
// k+1 and k+2 in flight in one launch; the in-line path only ever uses set 0).  Host-pointer
// frames of batch j are staged in slot j % kSlots and stay there until the launch that
// integrates them ends; the fourth slot lets the DMA of batch k+2 overlap launch k-1.
constexpr int kSets = 3;
constexpr int kSlots = 4;

// State common to the dense and hash handles.
struct Base {
    int device = 0;
    hipStream_t stream = nullptr;
    Vol vol{};
    Pool pool{};
    long long n_bricks = 0;
    // frames per launch (<= kMaxBatch, the kernels' Batch capacity): kMaxBatch for shards of a
    // multi-GPU volume, kFullBatch for whole volumes (set_batch; TSDF_BATCH overrides)
    int batch = kMaxBatch;
    int set_batch(int want);  // (tsdf_common.hip: also allocates buffer set 0's list)
    // frames a deferred per-frame batch collects (TSDF_DEFER) before it runs: 8 -- the host's
    // frame copies of the next batch overlap the ingest and integrate of this one at a finer
    // grain than a whole launch's 32 frames (TSDF_DEFER_FRAMES overrides)
    int defer_frames = 8;
    // deferred frames whose DMA is issued together while the batch fills (TSDF_DEFER_DMA_FRAMES)
    int dma_grain = 2;
    // RGB8 frames gathered in place by the integrate (frame_bufs) where the byte after a frame is
    // readable, instead of through the prep's RGBX copy (TSDF_RGB_DIRECT=0: always the copy)
    bool rgb_direct = true;
    // Texels (DK == 2 kernels, tsdf_device.h): the fused launches of u16 + RGB8 frames gather one
    // 8-byte (depth, colour) texel per voxel-step, written by their prep, where the handle holds at
    // least min_bricks bricks -- the integrate's gathers then outweigh the prep's 8 B per pixel.
    // Round 6 (profiles/r06_texel/), shards of 512^3 @ 8^3 bricks, texels against two gathers per
    // launch (scaling_sim, one box): dense whole -5 %, half -5 %, quarter -3 %, eighth +3 %; hash
    // whole -5 %, half -2 %, quarter +1 %, eighth +6 %.  So dense from 3 * 2^14 bricks (between an eighth and a
    // quarter), the hash from 3 * 2^15 (between a quarter and a half).
    // TSDF_TEXEL=0 / 1 forces it off / on.  texel_now: the batches being prepared carry texels.
    int texel_mode = -1;  // (-1: by the rule)
    bool texel_now = false;
    static constexpr long long kTexelMinBricksDense = 3ll << 14, kTexelMinBricksHash = 3ll << 15;
    bool texel_for(int dk, long long owned_bricks, long long min_bricks) const {
        if (dk != TSDF_DEPTH_U16_MM) return false;
        return texel_mode >= 0 ? texel_mode != 0 : owned_bricks >= min_bricks;
    }
    // deferred f64-metre frames that are all RN(k / 1000) staged as u16 millimetres (defer_push;
    // TSDF_DEFER_MM=0: as they come)
    bool defer_mm = true;
    // deferred batches still to be staged as f64 without trying u16 after a frame that was not
    // exact millimetres: a stream that mixes the two kinds would otherwise flush a u16 batch at
    // every such frame (batches of one or two frames; round-5 advisor finding)
    int mm_backoff = 0;
    static constexpr int kMmBackoff = 4;
    const char* call_color_end = nullptr;  // end of the current call's device colour array (begin_call)
    // Per-batch buffers of the CURRENT buffer set (use_set).
    float* pyr = nullptr;      // `batch` per-frame max-depth pyramids
    unsigned* rgbx = nullptr;  // `batch` per-frame packed RGB8 images
    int pyr_H = 0, pyr_W = 0;
    // per-batch list of (brick | frame mask << 24) kept by the cull: kMaxBatch sub-lists of
    // n_bricks entries, one per cost class (frames kept); count[c] = entries of class c (1..8)
    ListEntry* list = nullptr;
    unsigned int* count = nullptr;
    float* pyr_set[kSets] = {};
    unsigned* rgbx_set[kSets] = {};
    ListEntry* list_set[kSets] = {};
    unsigned int* count_set[kSets] = {};
    unsigned short* dmask_set[kSets] = {};
    int n_sets = 1;             // buffer sets allocated (kSets once the fused pipeline is used)
    int n_cu = 256;             // compute units of the device
    PyrLayout lay{};
    unsigned long long* stats = nullptr;  // kNStat x kStatSpread
    double* rcp = nullptr;                // reciprocal table (Vol::rcp)
    long long frames = 0;
    Profiler prof;
    // Host-pointer frames (frame ingest): the host copies each batch (with
    // several threads) into one of kSlots page-locked bounce slots, a copy stream DMAs it into
    // the matching device staging slot, and the compute stream integrates it -- while the host
    // already fills the next slot.
    hipStream_t cstream = nullptr;
    hipEvent_t ev_copied[kSlots] = {};  // slot's frames landed (copy stream)
    hipEvent_t ev_free[kSlots] = {};    // slot's last reader finished (compute stream)
    void* st_depth[kSlots] = {};
    void* st_color[kSlots] = {};
    size_t st_depth_bytes = 0, st_color_bytes = 0;
    unsigned short* dmask = nullptr;  // `batch` masked u16 depth images (TSDF_DEPTH_INVALID_65535)
    size_t dmask_px = 0;
    void* hst_depth[kSlots] = {};      // page-locked bounce slots (hipHostMalloc)
    void* hst_color[kSlots] = {};

    // Deferred single frames (TSDF_DEFER, the reference's one-integrate()-per-frame call
    // pattern): each call copies its frame straight into bounce slot `slot` and returns; every
    // defer_frames frames (or at any other call on the handle) the collected frames run as one
    // asynchronous batch -- temporal batching for per-frame callers, same results.
    struct Deferred {
        int n = 0, H = 0, W = 0, dk = 0, ck = 0, slot = -1;
        int dk_in = 0;   // the callers' depth kind (dk: as staged -- u16 for f64 metres that convert exactly)
        int copied = 0;  // frames whose DMA to the device staging slot is already issued
        double K[9];
        double T[16 * kMaxBatch];
        double ow[kMaxBatch];
    } dfr;
    int defer_next = 0;   // bounce slot of the next deferred batch
    int prestaged = -1;   // >= 0: the call's (single) batch already sits in this bounce slot
    int pre_copied = 0;   // ... and its first pre_copied frames are already on their way to the device
    bool defer_same(int dk, int ck, int H, int W, const double* K) const;
    // returns kDeferFlush when the frame cannot join the batch's kind: flush, then push it again
    int defer_push(const void* depth, int dk, const void* color, int ck, int H, int W,
                   const double* K, const double* T, double ow);
    static constexpr int kDeferFlush = 1;
    int stage_alloc(size_t dbytes, size_t cbytes);  // bounce + device staging slots (per frame)
    bool stage_fits(int dk, int ck, int H, int W) const {  // frames of this size need no reallocation
        return st_depth_bytes >= frame_bytes_depth(dk, H, W) * batch &&
               st_color_bytes >= frame_bytes_color(ck, H, W) * batch;
    }

    int init(int dev, const int64_t dims[3], const int64_t off[3], const float origin[3],
             double vs, double trunc);
    int use_sets(int n);  // allocate n buffer sets (1 or kSets)
    int cur_set = 0;
    void use_set(int s) {
        cur_set = s;
        pyr = pyr_set[s];
        rgbx = rgbx_set[s];
        list = list_set[s];
        count = count_set[s];
        dmask = dmask_set[s];
    }
    int sync_all();  // compute and copy streams (before reallocating per-batch buffers)
    int ensure_pyr(int H, int W);
    // Frame constants of frames [first, first+n) (n <= kMaxBatch) of a call, with the per-frame
    // buffers of the current set; host inputs are staged to the device through staging slot
    // `slot` (the work that reads them must follow on `stream`).
    int prepare_batch(Batch* bt, const void* depth, int dk, const void* color, int ck, int H,
                      int W, const double K[9], const double* Tinv, const double* ow,
                      double ow_default, int flags, int first, int n, int slot);
    // Around the batches of one integrate call: end_batch marks staging slot `slot` reusable
    // once the work issued so far on `stream` has finished.  begin_call / end_call bracket the
    // call (the caller's host arrays are read synchronously into the bounce slots, so nothing
    // of them is held past the call).
    int begin_call(const void* depth, size_t dbytes, const void* color, size_t cbytes, int flags);
    int end_batch(int flags, int slot);
    int end_call(int flags);
    int launch_prep(const Batch& bt, int dk, int ck, int W, int H, hipStream_t st);
    // Workgroups of the integrate kernel: as many as can be resident (occupancy x CUs), capped
    // by the work there can be (one brick per wave per round).
    unsigned grid_for(const void* kernel, int wg = kWG);
    // Workgroups of k_cull: one per superbrick (Vol::sb).
    unsigned cull_grid() const {
        long long n = 1;
        for (int a = 0; a < 3; ++a) n *= (vol.nb[a] + (1 << vol.sb[a]) - 1) >> vol.sb[a];
        return (unsigned)n;
    }
    // Superbricks per cull workgroup of a fused launch: 3 where the volume has >= 1024 superbricks
    // (the cull runs beside the integrate's tail: fewer slots taken, measured +2 % at 1, 2 and 4
    // ranks), 1 on smaller shards (the cull IS the launch's tail there: 3 cost 4.6 % on an eighth
    // shard); TSDF_CULL_G overrides.  And the cull workgroups of such a launch.
    int cull_g = 0;  // (0: by the rule)
    int cull_per_wg() const {
        if (cull_g > 0) return cull_g < kCullGMax ? cull_g : kCullGMax;
        return cull_grid() >= 1024 ? 3 : 1;
    }
    unsigned cull_grid_fused() const { return (cull_grid() + cull_per_wg() - 1) / cull_per_wg(); }
    int read_stats(tsdf_stats_t* out, int reset);
    // Vol::canon from the first n_vox voxels of the pool (after a set or an import; synchronous)
    int check_canon(long long n_vox);
    // a call whose frames may write non-canonical state (obs_weight != 1, folded f32 colour)
    void note_frames(int ck, const double* ow, int n, double ow_default) {
        if (ck != TSDF_COLOR_RGB8) vol.canon = 0;
        for (int i = 0; i < n; ++i)
            if ((ow ? ow[i] : ow_default) != 1.0) vol.canon = 0;
    }
    int set_profiling(int on);
    void release();
};

// An extracted mesh, in device memory (tsdf_mesh.hip).
struct Mesh {
    float* verts = nullptr;           // n_verts x 3 world coordinates
    float* normals = nullptr;         // n_verts x 3 unit normals (to positive tsdf)
    unsigned char* colors = nullptr;  // n_verts x 3 uint8 r, g, b
    int* faces = nullptr;             // n_tris x 3 vertex ids
    long long* keys = nullptr;        // n_verts global vertex keys ((x*Y + y)*Z + z)*3 + axis
    long long n_verts = 0, n_tris = 0;
    void release();
};
// The global x rows marching cubes runs over for one shard (tsdf_mesh.hip, Grid).
struct MeshDomain {
    int xlo = 0, xhi = 0;
    std::vector<int> row_map;               // [xhi - xlo]: local row, -2 - halo index, or -1
    std::vector<int> vrow_gx;               // vertex rows (local rows and cap rows), increasing x
    std::vector<unsigned char> vrow_cap;
};
// global_x > 0: the unsharded volume's x extent, halo rows given; 0: the shard alone
int mesh_domain(const Vol& v, long long global_x, const int64_t* halo_gx, long long n_halo, MeshDomain* d);
int mesh_halo_rows(const Vol& v, long long global_x, std::vector<long long>* out);
int extract_mesh(Base& B, const Pool& pool, Mesh& m, const MeshDomain& d, const float* ht, const float* hc);
int copy_mesh(Base& B, const Mesh& m, float* verts, float* normals, uint8_t* colors, int32_t* faces,
              int64_t* keys = nullptr);

// The state of a dense handle (tsdf_dense.hip), for the hash's densify into it.
Base* dense_base(tsdf_dense_t* d);

// end_call on every exit path of an integrate call (error returns included).
struct CallGuard {
    Base& b;
    int flags;
    bool done = false;
    CallGuard(Base& b_, int f) : b(b_), flags(f) {}
    int finish() {
        done = true;
        return b.end_call(flags);
    }
    ~CallGuard() {
        if (!done) (void)b.end_call(flags);
    }
};


int check_frame_args(const void* depth, int dk, const void* color, int ck, int H, int W,
                     const double* K, const double* Tinv);

}  // namespace tsdf
