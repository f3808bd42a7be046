// tsdf_device.h -- shared device code of the gfx950 TSDF fusion path.
//
// One integrate kernel serves both map stores:
//   * the dense grid (TSDFVolume, grid_fusion.py:19-320): brick b of the volume lives at
//     pool slot b (a direct-mapped brick table);
//   * the voxel hash (HashTable, hash_fusion.py:29-507): brick (bx,by,bz) lives at the pool
//     slot found by a wave-cooperative open-addressed probe of the block table.
// A workgroup culls 256 bricks (one per lane) against the frame, compacts the survivors with a
// wave ballot + LDS prefix sum, and its 4 waves then integrate those bricks, 8 voxels per lane.
//
// Numerics: every voxel follows the reference CPU path operation for operation (SURVEY §8(a)
// a3-a8; oracle/tsdf_oracle.c is the checker).  Compile with -ffp-contract=off: no
// multiply-add may be fused except the explicit fma() calls that restate OpenBLAS's dgemm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace tsdf {

constexpr int kBrickEdge = 8;
constexpr int kBrickVox = 512;      // 8^3 voxels; brick-local index = (x*8 + y)*8 + z
constexpr int kWG = 256;            // threads per workgroup (4 waves of 64)
constexpr int kPyrLevels = 6;       // max-depth pyramid levels 1..6 (2x2 .. 64x64 pixels)
constexpr int kStatSpread = 64;     // counters are spread over 64 words (no hot atomic word)
constexpr unsigned long long kEmpty = ~0ull;
constexpr unsigned long long kTomb = ~0ull - 1ull;

// ST_UNIQUE: voxels updated at least once by a launch's batch (each voxel's state is read and
// written once per batch however many of its frames update it: the roofline's state bytes)
enum Stat { ST_VOXELS = 0, ST_VISITED, ST_TOUCHED, ST_ALLOC, ST_PROBE, ST_LOOKUPS, ST_OVERFLOW,
            ST_PROBE_MAX, ST_BAD_ENTRY, ST_UNIQUE, kNStat };

// Volume geometry (by value in kernel arguments -> scalar registers).
struct Vol {
    int dims[3];    // voxels of this shard
    int off[3];     // global voxel index of local (0,0,0)
    int xstride;    // global x distance between local brick columns 2k and 2k+2 is 2*xstride (8:
                    // contiguous; 8*S: brick-column sharding over S ranks)
    int xodd;       // global x distance from local column 2k to 2k+1 (8: contiguous; xstride:
                    // plain cyclic; 8*(2S-1-2s): the mirrored pairs s, 2S-1-s of shard s)
    int sb[3];      // log2 superbrick edge in bricks per axis (sum 6: one wave = 64 bricks)
    int nb[3];      // bricks per axis (ceil(dims/8))
    int shard, n_shards;
    int canon;      // host-tracked: every stored weight is an integer >= 0 and every colour canonical
                    // (what integrate with obs_weight 1 and RGB8 colour writes); lets the integrate
                    // skip the per-load integrality checks (a max-range test remains)
    float origin[3];
    double vs, trunc;
    double rtrunc;  // RN(1 / trunc), from the host's IEEE division (Markstein quotient, below)
    const double* rcp;  // kRcpBig entries RN(1/n) in HBM (the first kRcpTab copied to LDS)
};

// Global x of local brick column c's first voxel, less off[0].
__host__ __device__ inline int col_gx(const Vol& v, int c) {
    return (c >> 1) * 2 * v.xstride + (c & 1) * v.xodd;
}

// Per-frame constants (by value).
struct Frame {
    double T[12];             // rows 0..2 of inv(cam_pose), row-major
    double fx, fy, cx, cy;    // f64(f32(K))  (cam2pix casts intr to float32, grid_fusion.py:190)
    double ow;                // obs_weight as a Python float (f64)
    double half_m;            // 0.5 - the fast pixel path's boundary margin (frame_margin)
    double Tf[8];             // the fast pixel path's rows: RN(T[0..3] * fx), RN(T[4..7] * fy)
    int zmin_hi;              // ... and its depth limit: high dword of zmin (fold_bound, host)
    float ow32;               // the same weight as NumPy's weak-scalar f32 (colour blend)
    int H, W;
    const void* depth;        // depth read by cull/integrate: u16 millimetres or f64 metres
    const void* depth_src;    // depth read by k_prep (== depth unless masking)
    unsigned short* depth_mask;  // TSDF_DEPTH_INVALID_65535: k_prep writes the masked u16 here
    const void* color;        // the caller's colour (RGB8 or folded f32)
    const unsigned* rgbx;     // RGB8 packed r | g<<8 | b<<16 per pixel (the prep writes it), or
                              // null: the integrate gathers the caller's RGB8 itself (frame_bufs)
    const float* pyr;         // max-depth pyramid (metres), levels 1..6 concatenated
    float planes[5][4];       // half-spaces n.q + d >= 0 containing every valid voxel, q = world
                              // point - eye (cull; camera-relative, so f32 stays accurate for
                              // volumes far from the world origin)
    double eye[3];            // camera centre in world coordinates
};

// Layout of a frame's max-depth pyramid (levels 1..kPyrLevels concatenated), the same for every
// frame of a batch.
struct PyrGeo {
    int off[kPyrLevels + 1];
    int w[kPyrLevels + 1];
    int h[kPyrLevels + 1];
};

// Up to kMaxBatch consecutive frames integrated by one launch (temporal batching: each voxel's
// updates are still applied frame by frame, in order, so results are those of one-by-one
// integration; the brick state is read and written once per batch instead of once per frame).
// 32 frames per launch (round 5: +2.8 % dense and +8.4 % hash on one GPU on equal frames, +2 % /
// +16 % on eighth shards against 16, profiles/r05_batch32/; round 4's 16 against 8: +6 % / +19 %,
// profiles/r04_e/); 16 and 8 remain build options (-DTSDF_MAX_BATCH=16)
#ifndef TSDF_MAX_BATCH
#define TSDF_MAX_BATCH 32
#endif
constexpr int kMaxBatch = TSDF_MAX_BATCH;
static_assert(kMaxBatch == 8 || kMaxBatch == 16 || kMaxBatch == 32, "frames per batch: 8, 16 or 32");
// Frames per launch of a whole (unsharded) volume; shards of a multi-GPU volume take kMaxBatch
// (Base::set_batch): a shard's launch is short, and its fixed costs -- dispatch, the end of the
// kernel, the cull / prep tail -- weigh more per frame.
#ifndef TSDF_FULL_BATCH
#define TSDF_FULL_BATCH TSDF_MAX_BATCH
#endif
constexpr int kFullBatch = TSDF_FULL_BATCH < kMaxBatch ? TSDF_FULL_BATCH : kMaxBatch;
// integrate_items / integrate_brick options (A/B builds)
#ifndef TSDF_XCD_DEAL  // deal list items to workgroups XCD by XCD (integrate_items): dense -1.5 %,
#define TSDF_XCD_DEAL 1  // hash -1 % per launch, hash eighth shard +3 % (profiles/r04_i/)
#endif
// (both measured neutral to -1.2 % at the driver window, profiles/r04_h2/ab.jsonl: off)
#ifndef TSDF_ITEM_PREFETCH  // take the next item before integrating the current one
#define TSDF_ITEM_PREFETCH 0
#endif
#ifndef TSDF_COLOR_U32  // fused launches on canonical volumes: colours held as u32 (integrate_brick CU;
#define TSDF_COLOR_U32 1  // round 5: dense -1.5 %, hash -1.5 % time per launch, profiles/r05_ab/)
#endif
// Per-set list counters (reset by the prep of the batch): word c = entries of cost class c
// (1..kMaxBatch); words kDoneWord / kDoneWordC = integrate and cull workgroups finished (fused hash
// launch; the launch counts on its cull's set, or on its integrate's set when it has no cull).
constexpr int kDoneWord = kMaxBatch + 8, kDoneWordC = kMaxBatch + 9;
constexpr int kCountWords = kMaxBatch + 16;
constexpr int kRcpTab = 4096;  // LDS table of RN(1/n), n < kRcpTab (32 KB per workgroup)
// The whole table in HBM (512 KB, L2-resident) for waves with a weight past the LDS part (long
// runs: weights pass 4079 after ~4300 frames of a room seen from inside); 65536 keeps every colour
// numerator w*c + c' below 2^24 (exact in f32).
constexpr int kRcpBig = 65536;

// w is an integer small enough that w + kMaxBatch indexes the reciprocal table
__device__ inline bool small_int(float w) {
    return w >= 0.0f && w < (float)(kRcpTab - kMaxBatch - 1) && w == truncf(w);
}
__device__ inline bool table_int(float w) {  // ... that indexes the HBM table
    return w >= 0.0f && w < (float)(kRcpBig - kMaxBatch - 1) && w == truncf(w);
}
// a canonical folded colour: an integer B*65536 + G*256 + R in [0, 2^24) (what integrate writes)
__device__ inline bool canon_color(float c) {
    return c >= 0.0f && c < 16777216.0f && c == truncf(c);
}
struct Batch {
    Frame f[kMaxBatch];
    PyrGeo pg;
    int n;
    int texel;  // the frames' rgbx buffers hold 8-byte depth + colour texels (DK == 2 kernels)
};

// A culled brick for the integrate: brick index (low 32 bits) | frames that kept it << 32.
typedef unsigned long long ListEntry;

// Brick storage: SoA pool of 512-voxel bricks.
struct Pool {
    float* tsdf;
    float* weight;
    float* color;
};

// Block table of the voxel hash (unused by the dense grid).
struct PoolState {
    long long pool_top;    // blocks handed out by the bump allocator
    long long free_count;  // blocks on the free list
    long long cursor;      // allocations made by the current launch
    long long n_overflow;  // bricks skipped for lack of space (re-run after growing)
    long long tombs;       // keys tombstoned since the table was last rebuilt (>= tombstones in it)
    long long n_inserted;  // blocks the fused launches' culls inserted since the last k_free_unused
};

// Pool state after launch `seq`, written by the committing thread into page-locked host memory
// (slot seq % kReports; `seq` stored last, system scope): asynchronous hash calls read it a
// couple of launches later to grow the pool / table before they fill up, and to detect
// skipped bricks, without a stream synchronisation per batch.
constexpr int kReports = 8;
struct PoolReport {
    long long pool_top, free_count, n_overflow;
    long long listed;  // bricks the launch's cull listed: a bound on the blocks one launch can allocate
    long long tombs;   // PoolState::tombs
    long long seq;     // launch number + 1 (0: slot never written)
};

struct Table {
    unsigned long long* keys;   // capacity slots; kEmpty / kTomb / packed brick key
    int* vals;                  // pool block of each slot
    unsigned long long* occ;    // [max_blocks][8] voxel-entry bits (word = z, bit = x*8+y)
    int* free_list;
    ListEntry* overflow;        // list entries skipped this launch
    PoolState* st;
    PoolReport* rb;             // kReports host-mapped report slots (nullptr: none)
    long long capacity;
    long long shard_cap;        // capacity at create: bucket-range ownership stays fixed across resizes
    long long max_blocks;
    const int* owned;           // bucket-range shards: the bricks this shard owns, increasing (else null)
    int n_owned;
    int* ins_list;              // fused launches: bricks their culls inserted (k_free_unused; ins_cap)
    long long ins_cap;
    int overflow_cap;
    int int_bits;               // 64: NumPy int64; 32: wrapping int32 (author's Windows run)
};

// hash_function (hash_fusion.py:182-190): ((x*P1) ^ (y*P2) ^ (z*P3)) floor-mod n.
template <bool POW2 = false>  // POW2: n is a power of two (the fused hash launch; no division code)
__host__ __device__ inline long long ref_hash(long long x, long long y, long long z, long long n,
                                              int int_bits) {
    const unsigned long long P1 = 73856093ull, P2 = 19349669ull, P3 = 83492791ull;
    long long h;
    if (int_bits == 32) {
        const int a = (int)(unsigned)((unsigned long long)x * P1);
        const int b = (int)(unsigned)((unsigned long long)y * P2);
        const int c = (int)(unsigned)((unsigned long long)z * P3);
        h = (long long)(a ^ b ^ c);
    } else {
        h = (long long)(((unsigned long long)x * P1) ^ ((unsigned long long)y * P2) ^
                        ((unsigned long long)z * P3));
    }
    // floor-mod; a power-of-two n (the bench's 2^22 buckets) by a mask -- the same residue for
    // negative h in two's complement -- instead of a 64-bit division (hundreds of VALU
    // instructions per brick in the integrate and the sharded cull)
    if (POW2 || (n & (n - 1)) == 0) return h & (n - 1);
    long long m = h % n;
    return m < 0 ? m + n : m;
}

// Shard owning home slot `home` of a table of `cap` slots (bucket ranges).
template <bool POW2 = false>
__host__ __device__ inline int shard_of(long long home, int n_shards, long long cap) {
    if (POW2 || (cap & (cap - 1)) == 0) return (int)((home * n_shards) >> (63 - __builtin_clzll((unsigned long long)cap)));
    return (int)((home * n_shards) / cap);
}

__host__ __device__ inline unsigned long long pack_key(int bx, int by, int bz) {
    return (unsigned long long)bx | ((unsigned long long)by << 21) | ((unsigned long long)bz << 42);
}

__device__ inline int lane_id() { return threadIdx.x & 63; }

// The integrate's per-step conditions as wave lane masks straight from the compares
// (llvm.amdgcn.fcmp / icmp: one v_cmp into an SGPR pair), combined by scalar ANDs / ORs, and turned
// back into a lane's condition by the inverse ballot (the mask itself drives v_cndmask and exec).
// A bool carried across basic blocks is otherwise rebuilt from a VGPR for every ballot of it
// (v_cndmask + v_cmp: ~14 VALU per wave-frame of the dense integrate).  The
// predicates are LLVM's: the C operators' semantics (a NaN compares false, != is unordered).
__device__ unsigned long long fcmp64_mask(double a, double b, int pred) __asm("llvm.amdgcn.fcmp.i64.f64");
__device__ unsigned long long fcmp32_mask(float a, float b, int pred) __asm("llvm.amdgcn.fcmp.i64.f32");
__device__ unsigned long long icmp32_mask(unsigned a, unsigned b, int pred) __asm("llvm.amdgcn.icmp.i64.i32");
constexpr int kCmpOGT = 2, kCmpOGE = 3, kCmpOLT = 4, kCmpUNE = 14, kCmpNE = 33, kCmpULT = 36, kCmpSGT = 38;
__device__ inline bool lane_in(unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// x = lane in m ? y : x, written in place (the register allocator otherwise gives the new value a
// register of its own and copies it back where the paths merge)
__device__ inline void sel_in_place(float& x, float y, unsigned long long m) {
    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(m));
}

// Shared table metadata (pool state, keys, slot values, entry masks) is read with agent-scope
// relaxed atomic loads: always a VECTOR load (global_load ... sc1).  A plain load from a
// wave-uniform address becomes an s_load through the scalar cache, which was measured to
// return stale pool counters right after the producing kernel.
template <typename T>
__device__ inline T coh_load(T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ inline void coh_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// World position of a global voxel index (vox2world, grid_fusion.py:170-181):
// f32( f64(origin_f32) + vs * f64(f32(idx)) ); idx < 2^24 so f32(idx) is exact.
__device__ inline double vox_world(float origin, double vs, int g) {
    return (double)(float)((double)origin + vs * (double)g);
}

// Conservative cull of one brick against one frame.  True = some voxel of the brick MAY pass the
// reference's masks (grid_fusion.py:273-290); a brick with a valid voxel is never dropped.  The
// brick's corner voxels are transformed (one corner in f64, the rest by f32 edge vectors) and
// projected in f32; every tolerance is covered by margins: 1 px on the bbox (projected bbox only
// when the whole brick is >= 0.2 m in front of the camera, where the f32 error is < 0.4 px),
// 0.1 mm on z <= 0, and 1 mm on the depth test against the max depth over the bbox.
struct BrickBox {
    double p0[3];  // world position of the low corner voxel (f64, exact lattice)
    float ext[3];  // (hi - lo) * vs per axis
    float ctr[3];  // centre of the voxel-centre box, relative to the frame's camera centre
    float rad;     // its half diagonal + 0.1 mm
};

// Box of the voxel centres of bricks [b, b + n) per axis (n = 1: one brick; larger: a superbrick,
// whose x extent spans the gaps between a cyclic shard's columns -- a superset, fine for culling).
__device__ inline BrickBox brick_box(const Vol& v, const double* eye, int bx, int by, int bz, int nx = 1,
                                     int ny = 1, int nz = 1) {
    const int bb[3] = {bx, by, bz}, nn[3] = {nx, ny, nz};
    BrickBox r;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int lo = bb[a] * kBrickEdge;
        const int hi = min(lo + nn[a] * kBrickEdge - 1, v.dims[a] - 1);
        // global indices of the low / high corner (x: local brick column -> global column)
        const int glo = (a == 0) ? col_gx(v, bb[0]) : lo;
        const int ghi = (a == 0) ? col_gx(v, hi >> 3) + (hi & 7) : hi;
        r.p0[a] = (double)v.origin[a] + v.vs * (double)(glo + v.off[a]);
        r.ext[a] = (float)(v.vs * (double)(ghi - glo));
        r.ctr[a] = (float)(r.p0[a] + 0.5 * v.vs * (double)(ghi - glo) - eye[a]);
    }
    r.rad = 0.5f * sqrtf(r.ext[0] * r.ext[0] + r.ext[1] * r.ext[1] + r.ext[2] * r.ext[2]) + 1e-4f;
    return r;
}

__device__ inline bool cull_brick(const Vol& v, const Frame& fr, const PyrGeo& pg, const BrickBox& bb) {
    // early out: the brick's bounding sphere entirely outside one of the frustum half-spaces
    // (z > 0 and -0.5 <= u < W - 0.5, -0.5 <= v < H - 0.5, each widened by 1 px)
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const float* q = fr.planes[i];
        if (q[0] * bb.ctr[0] + q[1] * bb.ctr[1] + q[2] * bb.ctr[2] + q[3] < -bb.rad) return false;
    }
    const double* T = fr.T;
    float c0[3], d[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        c0[r] = (float)(T[4 * r + 0] * bb.p0[0] + T[4 * r + 1] * bb.p0[1] + T[4 * r + 2] * bb.p0[2] + T[4 * r + 3]);
#pragma unroll
        for (int a = 0; a < 3; ++a) d[r][a] = (float)T[4 * r + a] * bb.ext[a];
    }
    const float fx = (float)fr.fx, fy = (float)fr.fy, cx = (float)fr.cx, cy = (float)fr.cy;
    float zmin = 3e38f, zmax = -3e38f, umin = 3e38f, umax = -3e38f, vmin = 3e38f, vmax = -3e38f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float q[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            q[r] = c0[r] + ((c & 1) ? d[r][0] : 0.0f) + ((c & 2) ? d[r][1] : 0.0f) + ((c & 4) ? d[r][2] : 0.0f);
        zmin = fminf(zmin, q[2]);
        zmax = fmaxf(zmax, q[2]);
        const float iz = __builtin_amdgcn_rcpf(fmaxf(q[2], 1e-6f));
        const float u = fx * q[0] * iz + cx, w = fy * q[1] * iz + cy;
        umin = fminf(umin, u); umax = fmaxf(umax, u);
        vmin = fminf(vmin, w); vmax = fmaxf(vmax, w);
    }
    if (zmax < -1e-4f) return false;  // every voxel has z <= 0
    int u0 = 0, u1 = fr.W - 1, v0 = 0, v1 = fr.H - 1;
    if (zmin > 0.2f) {  // whole brick well in front of the camera: projected hull is convex
        const float fu0 = floorf(umin) - 1.0f, fu1 = ceilf(umax) + 1.0f;
        const float fv0 = floorf(vmin) - 1.0f, fv1 = ceilf(vmax) + 1.0f;
        if (fu1 < 0.0f || fv1 < 0.0f || fu0 > (float)(fr.W - 1) || fv0 > (float)(fr.H - 1)) return false;
        u0 = (int)fmaxf(fu0, 0.0f); u1 = (int)fminf(fu1, (float)(fr.W - 1));
        v0 = (int)fmaxf(fv0, 0.0f); v1 = (int)fminf(fv1, (float)(fr.H - 1));
    }
    // max depth over the bbox from the smallest pyramid level where it spans <= 4x4 texels (16
    // independent predicated loads); a bbox wider than that at the coarsest level (a box very
    // close to the camera) is kept without a depth test
    int L = 1;
    while (L < kPyrLevels && (((u1 >> L) - (u0 >> L)) > 3 || ((v1 >> L) - (v0 >> L)) > 3)) ++L;
    const float need = zmin - (float)v.trunc - 1e-3f;
    const int tx0 = u0 >> L, tx1 = u1 >> L, ty0 = v0 >> L, ty1 = v1 >> L;
    if (tx1 - tx0 > 3 || ty1 - ty0 > 3) return true;
    const float* lvl = fr.pyr + pg.off[L];
    const int wl = pg.w[L];
    float dmax = 0.0f;
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx)
            if (ty0 + dy <= ty1 && tx0 + dx <= tx1) dmax = fmaxf(dmax, lvl[(ty0 + dy) * wl + tx0 + dx]);
    return dmax > 0.0f && dmax >= need;
}

// Take one block from the pool: the free list first, then the bump region.  `cursor` counts
// this launch's allocations; k_commit folds it into free_count / pool_top afterwards, so both
// stay constant while the launch runs.  Returns -2 when the pool is exhausted.
__device__ inline int pool_alloc(const Table& t) {
    const long long c = (long long)atomicAdd((unsigned long long*)&t.st->cursor, 1ull);
    const long long nf = coh_load(&t.st->free_count);
    const long long b = (c < nf) ? (long long)coh_load(&t.free_list[nf - 1 - c])
                                 : coh_load(&t.st->pool_top) + (c - nf);
    return (b < t.max_blocks) ? (int)b : -2;
}

// Wave-cooperative lookup-or-insert of a brick key (64 slots per probe step, one CAS by one
// lane).  Returns the pool block (>= 0), or -1 when the table/pool is full.  Sets is_new.
// Keys are only ever written by CAS, so a stale plain read can only cost a retry.
__device__ inline int table_find_or_insert(const Table& t, unsigned long long key, long long home,
                                           bool insert, bool& is_new, long long& slot_out,
                                           long long& probe) {
    const int lane = lane_id();
    is_new = false;
    long long pos = home;
    long long tomb = -1;
    int blk = -1;  // block allocated for this key (kept across CAS retries)
    for (long long scanned = 0; scanned < t.capacity + 64;) {
        long long s = pos + lane;
        if (s >= t.capacity) s -= t.capacity;
        if (s >= t.capacity) s %= t.capacity;
        // the slot values load beside the keys (one memory latency per probe step instead of two);
        // a key found here was inserted by an earlier launch or by this wave, so its value is set
        const unsigned long long kk = coh_load(&t.keys[s]);
        const int vv = coh_load(&t.vals[s]);
        const unsigned long long hit = __ballot(kk == key);
        if (hit) {
            const int l = __ffsll((long long)hit) - 1;
            slot_out = __shfl(s, l);
            probe = scanned + l;
            return __shfl(vv, l);
        }
        const unsigned long long emp = __ballot(kk == kEmpty);
        unsigned long long tm = __ballot(kk == kTomb);
        if (emp) tm &= (emp & (~emp + 1)) - 1;  // tombstones before the first empty slot only
        if (tomb < 0 && tm) tomb = __shfl(s, __ffsll((long long)tm) - 1);
        if (emp) {
            if (!insert) return -1;
            const int le = __ffsll((long long)emp) - 1;
            const long long target = tomb >= 0 ? tomb : __shfl(s, le);
            const unsigned long long expect = tomb >= 0 ? kTomb : kEmpty;
            int ok = 0;
            if (lane == 0) {
                if (blk < 0) blk = pool_alloc(t);
                if (blk >= 0) {
                    const unsigned long long old = atomicCAS(&t.keys[target], expect, key);
                    if (old == expect) {
                        coh_store(&t.vals[target], blk);
                        ok = 1;
                    } else if (old == key) {
                        ok = 2;  // a stale read hid our own key: it is there already
                    }
                }
            }
            blk = __shfl(blk, 0);
            ok = __shfl(ok, 0);
            if (blk == -2) return -1;  // pool exhausted
            if (ok == 1) {
                is_new = true;
                slot_out = target;
                probe = scanned + ((target - pos + t.capacity) % t.capacity);
                return blk;
            }
            if (ok == 2) {  // never happens with coherent reads; keep the spare block unused
                slot_out = target;
                probe = scanned + ((target - pos + t.capacity) % t.capacity);
                return coh_load(&t.vals[target]);
            }
            // another wave took that slot: continue probing just past it
            scanned += (target - pos + t.capacity) % t.capacity + 1;
            pos = target + 1;
            if (pos >= t.capacity) pos -= t.capacity;
            tomb = -1;
            continue;
        }
        pos += 64;
        if (pos >= t.capacity) pos -= t.capacity;
        scanned += 64;
    }
    return -1;  // table full
}


// Depth in metres at pixel p exactly as NumPy computes it: u16 mm -> astype(float) / 1000.
// (grid_demo1.py:81-82).  For u16 input the quotient is fma(m, C_HI, m * C_LO) with the two-term
// 1/1000 = C_HI + C_LO, which equals RN(m / 1000) for every m in [0, 65535] (checked
// exhaustively: tools/check_depth_conversion.c) -- one f64 multiply fewer than q = m * 0.001 plus
// an FMA correction.  depth_raw issues the u16 load; depth_m converts.  For f64 depth (DK == 1)
// depth_raw is unused and depth_m loads.
// The per-step gathers go through structured buffer descriptors (stride = texel size, idxen):
// the hardware scales the pixel index (p < 2^28, check_frame_args), so there is no shift or
// 64-bit address arithmetic per gather.  num_records = pixels of the image; non-candidate steps
// read pixel 0.
__device__ unsigned short buf_ld_u16(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                                     int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.i16");
__device__ unsigned buf_ld_u32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                               int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ double buf_ld_f64(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                             int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.f64");
constexpr int kBufDword3 = 0x00020000;  // gfx9 untyped buffer access
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ u32x2 buf_ld_v2u32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                              int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v2i32");
// DK == 2 ("texels"): u16 millimetre depth + RGB8 gathered as ONE 8-byte texel per pixel (depth,
// r | g<<8 | b<<16), which the fused launch's prep writes into the frame's rgbx buffer (Batch::texel)
// -- one gather per voxel-step instead of two (round 6: dense -4.7 % per launch; the prep's 8 B per
// pixel then costs more than it saves on eighth shards, so the host picks it by the handle's
// bricks, Base::texel_for)
struct FrameBufs {
    __amdgpu_buffer_rsrc_t depth, color;
};
template <int DK, int CK>
__device__ inline FrameBufs frame_bufs(const Frame& fr) {
    const int n = fr.W * fr.H;
    FrameBufs b;
    if (DK == 2) {
        static_assert(DK != 2 || CK == 0, "texels: RGB8 colour");
        b.depth = b.color = __builtin_amdgcn_make_buffer_rsrc((void*)fr.rgbx, 8, n, kBufDword3);
        return b;
    }
    b.depth = __builtin_amdgcn_make_buffer_rsrc((void*)fr.depth, DK == 0 ? 2 : 8, n, kBufDword3);
    // RGB8 (CK == 0): a 4-byte load at pixel p of a 3-byte-stride structured buffer returns r, g, b in
    // bytes 0-2 (the integrate decodes those three; the range check is on the pixel index), so the
    // caller's frame is gathered as it lies -- provided the byte after its last pixel is readable
    // (prepare_batch: the call's array or the padded staging slot goes on); otherwise the prep's
    // packed RGBX copy (round 5: dense +1.0 %, hash +1.6 %, eighth shards +2.9 % / +5.8 %,
    // profiles/r05_rgb_direct/)
    if (CK == 0 && !fr.rgbx) b.color = __builtin_amdgcn_make_buffer_rsrc((void*)fr.color, 3, n, kBufDword3);
    else b.color = __builtin_amdgcn_make_buffer_rsrc((void*)(CK == 0 ? (const void*)fr.rgbx : fr.color), 4, n, kBufDword3);
    return b;
}
template <int DK>
__device__ inline unsigned depth_raw(const FrameBufs& fb, unsigned p) {
    return DK == 0 ? (unsigned)buf_ld_u16(fb.depth, (int)p, 0, 0, 0) : 0u;  // (DK 2: the texel's)
}
template <int DK>
__device__ inline double depth_m(const FrameBufs& fb, unsigned p, unsigned raw) {
    if (DK != 1) {  // two-term 1/1000 = C_HI + C_LO: exact for every u16 (tools/check_depth_conversion.c)
        const double m = (double)raw;
        return fma(m, 0.001, m * -2.0858186326137145e-20);
    }
    return buf_ld_f64(fb.depth, (int)p, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// Reciprocal of z for the fast pixel path: the bare v_rcp_f64, accurate to 2^-24.4 relative
// (random z in [1e-3, 1e3] and a 2^28-point mantissa sweep: tools/gpu/rcp_probe.hip), so
// u = (x*fx)*rz + cx lies within |u - cx| * 2^-24.3 of the reference's (x*fx)/z + cx (< 3e-5 px
// for 640x480).  Steps whose u is within frame_margin of a rounding boundary (or not finite) are recomputed with the reference's own division (a Newton-refined reciprocal
// with a 1e-9 px margin ran 2.6 % slower: the two FMAs cost more than the extra slow steps).
// ---------------------------------------------------------------------------------------------
// RN(a / b) given y = RN(1 / b): Markstein's correction step.  q0 = RN(a*y) is within 1 ulp
// of a/b, r = a - b*q0 is exact with an FMA, and RN(q0 + r*y) is then the correctly rounded
// quotient (Markstein 1990; Muller et al., Handbook of Floating-Point Arithmetic, "Markstein's
// theorem"), barring under/overflow, which the TSDF ranges exclude.  tests/test_numerics_cpu.py
// re-checks it on the kernels' operand ranges.
__device__ inline double div_rn(double a, double b, double y) {
    const double q0 = a * y;
    const double r = fma(-q0, b, a);
    return fma(r, y, q0);
}

// The same in f32 (y = RN32(1/b)); operands here are integers, so never subnormal.
__device__ inline float div_rn32(float a, float b, float y) {
    const float q0 = a * y;
    const float r = fmaf(-q0, b, a);
    return fmaf(r, y, q0);
}

// Two f32 lanes per VGPR pair: the packed ALU (v_pk_fma_f32, v_pk_mul_f32, v_pk_add_f32).
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ inline f2 rint2(f2 a) { return f2{rintf(a.x), rintf(a.y)}; }
__device__ inline f2 div_rn32x2(f2 a, f2 b, f2 y) {  // div_rn32 on both lanes
    const f2 q0 = a * y;
    const f2 r = pk_fma(-q0, b, a);
    return pk_fma(r, y, q0);
}

// The fast path's pixel error is < |u - c| * 2^-24.3 (the bare reciprocal), and wherever the
// boundary test matters |u - c| <= max(W, H) + max(|cx|, |cy|) -- a step closer than this margin to
// a rounding boundary takes the exact path.  1e-4 px covers images up to ~1000 px; larger ones
// scale it.  Host-side: stored per frame as half_m = 0.5 - margin.
inline double frame_margin(int W, int H, double cx, double cy) {
    const double span = (double)(W > H ? W : H) + fmax(fabs(cx), fabs(cy));
    return fmax(1e-4, 1e-7 * span);
}

// The fast path folds fx, fy and the translation into its rows: X = fma(Tf2, pz, fma(Tf1, py,
// fma(Tf0, px, Tf3))) with Tf = RN(T * f) -- four roundings, each within 2^-53 of its operands'
// magnitudes, so |X - f * x| <= E = 8 * 2^-53 * f * (|T0| X + |T1| Y + |T2| Z + |T3|) for world
// coordinates bounded by (X, Y, Z) (a factor 2 of slack).  Its pixel error E / z stays below a
// quarter of the margin where z > zmin = 4 E / margin.  Returns zmin (host).
inline double fold_bound(const double* T, double fx, double fy, const double wmax[3], double margin) {
    double e = 0.0;
    for (int r = 0; r < 2; ++r) {
        const double* t = T + 4 * r;
        const double s = fabs(t[0]) * wmax[0] + fabs(t[1]) * wmax[1] + fabs(t[2]) * wmax[2] + fabs(t[3]);
        e = fmax(e, 8.0 * 0x1p-53 * (r == 0 ? fx : fy) * s);
    }
    return 4.0 * e / margin;
}

// v_cvt_i32_f64 clamps out-of-range inputs to INT_MIN / INT_MAX (a C cast would be undefined
// there, so the instruction is named directly)
__device__ inline int cvt_i32_sat(double x) {
    int r;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ inline double readlane_f64(double x, int l) {
    const unsigned long long u = __double_as_longlong(x);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | lo);
}

// ---------------------------------------------------------------------------------------------
// Per-brick integrate, one wave, over the frames of a batch in which the cull kept the brick.
// Lane (x,y) = (lane>>3, lane&7) owns the z-column of the brick and walks z = 0..7: the x/y part
// of the camera transform is computed once per column, and the brick-local layout [x][y][z]
// makes the column 32 contiguous bytes per field, so the state moves with 16-byte loads/stores
// (a wave: one contiguous 2 KB segment per field).  The state stays in registers across the
// batch's frames (loaded at its first use, stored once at the end); within a frame the 8 z-steps
// go through the phases together (project -> gather depth -> test -> colour -> update) to keep
// many loads in flight per lane.
// ---------------------------------------------------------------------------------------------
// NZ = 8: one wave per brick (lane = (x, y) column, 8 z-steps).  NZ = 4 (dense only): two waves
// per brick, one per z-half (zoff = 0 or 4) -- twice the waves for small culled lists (sharded
// volumes), where one brick per wave leaves SIMDs idle, and half the per-lane registers.

#ifdef TSDF_DIAG
// Diagnostic builds only (tools/gpu/diag_pairs.py): how often the integrate's paths run, summed over
// launches -- 0 part-frames projected, 1 ... with an update, 2 steps whose pixel was redone with the
// reference's division, 3 part-frames with such a step, 4 free-space skips of the update's
// quotients, 5 part-frames on the exact (non-canonical) path
__device__ unsigned long long g_ddiag[8];
#define TSDF_DDIAG(i) (lane_id() == 0 ? (void)atomicAdd(&g_ddiag[i], 1ull) : (void)0)
#else
#define TSDF_DDIAG(i) ((void)0)
#endif

// Phases 1-3 of one frame for one part (z-steps zoff .. zoff+NZ-1 of a lane's column): project,
// gather, depth / truncation test.  ok[k]: step k updates its voxel; fills the packed colour
// texels and depth - z of every step (dist_of gives the clamped distance; the integrate computes
// it only where a voxel needs it).  The per-step conditions stay booleans (lane
// masks in SGPR pairs): their combinations and wave ballots are scalar instructions, not VALU.
template <int DK, int CK, int NZ>
__device__ __forceinline__ void project_part(double trunc, const Frame& fr, double px, double py,
                                             const double* pzs, double pz_l, int zoff, unsigned long long colm,
                                             int nz, unsigned (&cpx)[NZ], double (&diff)[NZ],
                                             unsigned long long (&okm)[NZ]) {
    constexpr int kPz = NZ < 8 ? NZ : 1;
    // the z term of OpenBLAS's dgemm chain (grid_fusion.py:363-368): exact, it feeds the depth test
    const double a2 = fma(fr.T[9], py, fr.T[8] * px);
    // the pixel's numerators with fx, fy and the translation folded in (fast path only: their
    // error is bounded on the host, fold_bound, and covered by the boundary margin)
    const double b0 = fma(fr.Tf[1], py, fma(fr.Tf[0], px, fr.Tf[3]));
    const double b1 = fma(fr.Tf[5], py, fma(fr.Tf[4], px, fr.Tf[7]));
    // phase 1: project (grid_fusion.py:262-277).  Straight-line code over the z-steps (no
    // per-step branches) so the compiler can interleave their f64 chains; the rare steps whose
    // pixel lies within frame_margin of a rounding boundary are redone exactly afterwards.
    // the pixel indices leave the f64 domain at once (saturating v_cvt_i32_f64: out-of-range
    // values clamp to INT_MIN / INT_MAX and fail the unsigned bounds test below), which keeps
    // two f64 per step out of the registers live across the gathers
    double zc[NZ];
    int iu[NZ], iv[NZ];
    unsigned long long in[NZ], slow[NZ], any_slow = 0;  // lane masks (fcmp64_mask)
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        const double pz = NZ < 8 ? pzs[k % kPz] : readlane_f64(pz_l, k + zoff);
        zc[k] = fr.T[11] + fma(fr.T[10], pz, a2);  // fma(T3, 1, s) == T3 + s
    }
    double rzs[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) rzs[k] = __builtin_amdgcn_rcp(zc[k]);  // v_rcp_f64, see frame_margin
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        const double pz = NZ < 8 ? pzs[k % kPz] : readlane_f64(pz_l, k + zoff);
        const double z = zc[k], rz = rzs[k];
        // X*rz + cx with X = x*fx up to the folding error: within |u - cx| * 2^-24.3 + E/z of
        // the reference's (x*fx)/z + cx, inside the frame_margin boundary margin below where
        // z > zmin (E/z < margin/4; the high-dword integer test is a conservative z > zmin)
        const double sx = fma(fma(fr.Tf[2], pz, b0), rz, fr.cx), sy = fma(fma(fr.Tf[6], pz, b1), rz, fr.cy);
        const double ux = rint(sx), uy = rint(sy);
        // (a NaN fails both tests and takes the exact path; far-out |s| may round differently
        // but is invalid either way)
        // fine: z > zmin (so z > 0; the high-dword test passes a positive NaN, which then fails
        // the pixel tests) and both pixel coordinates clear of a rounding boundary.  The other
        // steps of the column (rare: near a boundary, at or behind the camera plane) take the
        // z > 0 test and, where it holds, the exact path below
        const unsigned long long fine = fcmp64_mask(fabs(sx - ux), fr.half_m, kCmpOLT) &
                                        fcmp64_mask(fabs(sy - uy), fr.half_m, kCmpOLT) &
                                        icmp32_mask((unsigned)(__double_as_longlong(z) >> 32), (unsigned)fr.zmin_hi, kCmpSGT);
        const unsigned long long col = k < nz ? colm : 0ull;
        in[k] = col & fine;
        iu[k] = cvt_i32_sat(ux);
        iv[k] = cvt_i32_sat(uy);
        slow[k] = col & ~fine;  // (z > 0 still to test)
        any_slow |= slow[k];
    }
    TSDF_DDIAG(0);
    if (any_slow) {
        TSDF_DDIAG(3);
        const double a0 = fma(fr.T[1], py, fr.T[0] * px);  // the reference's x / y chains
        const double a1 = fma(fr.T[5], py, fr.T[4] * px);
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            slow[k] &= fcmp64_mask(zc[k], 0.0, kCmpOGT);
            in[k] |= slow[k];
            if (!slow[k] || !lane_in(slow[k])) continue;
            TSDF_DDIAG(2);
            const double pz = NZ < 8 ? pzs[k % kPz] : readlane_f64(pz_l, k + zoff);
            const double x = fr.T[3] + fma(fr.T[2], pz, a0);
            const double y = fr.T[7] + fma(fr.T[6], pz, a1);
            iu[k] = cvt_i32_sat(rint((x * fr.fx) / zc[k] + fr.cx));  // the reference's own operation order
            iv[k] = cvt_i32_sat(rint((y * fr.fy) / zc[k] + fr.cy));
        }
    }
    unsigned long long cand[NZ];
    unsigned pix[NZ];
    const int W = fr.W, H = fr.H;
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        // unsigned bounds on the saturated indices (they come from integral, non-NaN values
        // wherever z > 0: the exact path yields NaN only for a non-finite pose, whose z --
        // np.linalg.inv: all NaN -- fails z > 0)
        cand[k] = in[k] & icmp32_mask((unsigned)iu[k], (unsigned)W, kCmpULT) &
                  icmp32_mask((unsigned)iv[k], (unsigned)H, kCmpULT);
        pix[k] = lane_in(cand[k]) ? __umul24((unsigned)iv[k], (unsigned)W) + (unsigned)iu[k] : 0u;  // v_mad_u32_u24
    }
    // phase 2: gather depth and colour for every step at once, before the depth test, so
    // all the gathers share one memory latency (non-candidates read pixel 0, discarded).  The
    // scheduling barrier keeps the compiler from sinking each load next to its use, which
    // under the VGPR budget it otherwise does, serialising the latencies.
    const FrameBufs fb = frame_bufs<DK, CK>(fr);
    unsigned draw[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        if (DK == 2) {
            const u32x2 t = buf_ld_v2u32(fb.depth, (int)pix[k], 0, 0, 0);
            draw[k] = t.x;
            cpx[k] = t.y;
        } else {
            draw[k] = depth_raw<DK>(fb, pix[k]);
            cpx[k] = buf_ld_u32(fb.color, (int)pix[k], 0, 0, 0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    double dep[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) dep[k] = depth_m<DK>(fb, pix[k], draw[k]);
    // phase 3: depth / truncation test and distance (grid_fusion.py:278-286)
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        diff[k] = dep[k] - zc[k];
        // u16: RN(m / 1000) > 0 iff m > 0
        const unsigned long long dpos = DK != 1 ? icmp32_mask(draw[k], 0u, kCmpNE) : fcmp64_mask(dep[k], 0.0, kCmpOGT);
        okm[k] = cand[k] & dpos & fcmp64_mask(diff[k], -trunc, kCmpOGE);
    }
}

// np.minimum(1, (depth - z) / trunc) (grid_fusion.py:284-286; the quotient is never NaN)
__device__ inline double dist_of(double trunc, double rtrunc, double diff) {
    return fmin(div_rn(diff, trunc, rtrunc), 1.0);
}

// Hash z-half waves (NZ = 4, the fused hash launch; round 5).  The cull that lists a brick one
// launch ahead also finds or inserts its block (cull_find_or_insert: a new block is initialised to
// (1, 0, 0) with no entries by the cull's wave) and leaves it in the brick's claim word of the batch
// (res[b]), or kResFail when the table or pool is full.  So both halves of a brick start at once
// from their block and run like the dense grid's z-halves -- no lookup, no insert, no waiting on the
// other half inside the integrate (round 4's claim / wait protocol cost the inserting launch 21 %).
// A block the batch then leaves without an entry is freed at the end of the call (k_free_unused),
// so the table holds the reference's keys.  A kResFail brick goes whole to the host's exact re-run
// (listed by its z-low wave).
constexpr int kResFree = -1, kResFail = -3;

// CU (u32 colour registers): the launch's volume is canonical (Vol::canon, host-checked), so every
// colour the wave holds is an integer B*65536 + G*256 + R; it is held as that u32 between load and
// store instead of as its f32, which the fast update decodes with byte conversions and encodes with
// v_cvt_pk_u8_f32 (round to nearest even and clamp: the rint of the reference's blend, whose result
// is <= 255) -- four VALU instructions fewer per step pair than through the f32.
template <bool HASH, int DK, int CK, bool OW1, int NZ, bool CU = false>
__device__ inline void integrate_brick(const Vol& v, const Batch& bt, const Pool& pool,
                                       const Table& tab, ListEntry entry, int zoff,
                                       unsigned long long* s_stat, const double* s_rcp,
                                       unsigned& nupd, unsigned& nuniq, int* res = nullptr) {
    static_assert(!CU || (CK == 0 && OW1), "u32 colour registers: RGB8 frames, obs_weight 1");
    // nupd: the wave's voxel updates, accumulated over its items (scalar popcounts of the step
    // masks; integrate_list adds it to the statistics once per wave); nuniq: the voxels among them
    // updated at least once in the batch (popcounts of the OR of each step's masks over the frames)
    static_assert(NZ == 8 || NZ == 4, "z-parts of 8 or 4 steps");
    constexpr bool kHalfHash = HASH && NZ == 4;  // (requires res)
    const int lane = lane_id();
    // (wave-uniform: scalar registers, so the frame loop below walks the mask's set bits with
    // scalar instructions)
    const int b = __builtin_amdgcn_readfirstlane((int)(entry & 0xFFFFFFFFull));
    const unsigned fmask = __builtin_amdgcn_readfirstlane((unsigned)(entry >> 32));
    // the volume fields the frame loop reads, once per item (v is re-read per item through an
    // opaque pointer, item_vol: its other fields are not held across the frame loop)
    const double trunc = v.trunc, rtrunc = v.rtrunc;
    const double* const rcp_hbm = v.rcp;
    const bool canon = CU || v.canon != 0;
    const int nb12 = v.nb[1] * v.nb[2];
    if (b >= v.nb[0] * nb12) {  // never for a list k_cull wrote; guards the pool against bad input
        if (lane == 0) atomicAdd(&s_stat[ST_BAD_ENTRY], 1ull);
        return;
    }
    const int bx = b / nb12;
    const int rem = b - bx * nb12;
    const int by = rem / v.nb[2];
    const int bz = rem - by * v.nb[2];
    const int lx = bx * kBrickEdge + (lane >> 3);
    const int ly = by * kBrickEdge + (lane & 7);
    const unsigned long long colm = __ballot(lx < v.dims[0] && ly < v.dims[1]);  // the item's columns inside
    const int nz = min(kBrickEdge, v.dims[2] - bz * kBrickEdge) - zoff;  // valid steps of this part
    // vox2world (grid_fusion.py:170-181); lanes 0..7 compute the brick's 8 z coordinates
    const double px = vox_world(v.origin[0], v.vs, v.off[0] + col_gx(v, bx) + (lane >> 3));
    const double py = vox_world(v.origin[1], v.vs, v.off[1] + ly);
    const double pz_l = vox_world(v.origin[2], v.vs, v.off[2] + bz * kBrickEdge + (lane & 7));  // lane k: z = k
    // z-part waves (NZ = 4, dense): this part's z coordinates read out of the lanes once per item
    // (+1.5 %); with NZ = 8 the hash kernel has no registers to spare and reads them per frame
    constexpr int kPz = NZ < 8 ? NZ : 1;
    double pzs[kPz];
#pragma unroll
    for (int k = 0; k < kPz; ++k) {
        pzs[k] = readlane_f64(pz_l, k + zoff);
        // held in VGPRs: an FMA with a frame's scalar operand could not take it from SGPRs (one
        // scalar operand per VOP3), so the projection would copy it back per frame
        if (NZ < 8) asm("" : "+v"(pzs[k]));
    }

    // the brick's storage: dense brick b, or its hash pool block (wave-uniform; 32-bit for the hash,
    // where it is one register fewer across the frame loop -- the dense kernel measured faster as is)
    typename std::conditional<HASH, int, long long>::type blk = HASH ? -1 : b;  // (dense: its brick)
    bool is_new = false;
    bool upd = false;  // a frame of the batch updates this part (wave-uniform)
    if constexpr (kHalfHash) {
        // the cull's block (written by the previous launch), or kResFail
        const int cur = __builtin_amdgcn_readfirstlane(res[b]);
        if (cur == kResFail) {  // no room: the whole brick waits for the host's exact re-run
            if (zoff == 0 && lane == 0) {
                const unsigned long long o = atomicAdd((unsigned long long*)&tab.st->n_overflow, 1ull);
                if ((long long)o < tab.overflow_cap) tab.overflow[o] = entry;
                atomicAdd(&s_stat[ST_OVERFLOW], 1ull);
            }
            return;
        }
        if (cur < 0 || cur >= tab.max_blocks) {  // never: the cull writes a block or kResFail
            if (lane == 0) atomicAdd(&s_stat[ST_BAD_ENTRY], 1ull);
            return;
        }
        blk = cur;
    }
    float ws[NZ], ts[NZ], cs[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        ws[k] = 0.0f;
        ts[k] = 1.0f;
        cs[k] = 0.0f;
    }
    // 16-B halves of this lane's column held in registers (half h: z 4h .. 4h+3 of the part); a
    // half of a block this launch inserted starts at (1, 0, 0): nothing to load.  Every half held
    // is stored at the end (a changed half, or -- a new hash block -- its init).  Lane masks.
    constexpr int kH = NZ / 4;
    unsigned long long loaded[kH];  // lane masks
#pragma unroll
    for (int h = 0; h < kH; ++h) loaded[h] = 0;
    // voxels updated by any frame of the batch (entry bits of the hash, ST_UNIQUE): per z-step,
    // the OR of the step masks' ballots -- scalar registers and scalar ORs, no per-lane VGPR bit field
    unsigned long long touched[NZ] = {};
    bool w_small = true;   // all loaded weights are integers that stay < kRcpTab in this batch
    bool w_table = true;   // ... < kRcpBig
    bool c_canon = true;   // all loaded colours are canonical (canon_color)
    // the wave-uniform fast-path choices below, refreshed whenever the wave loads state
    bool fast_t = OW1 && s_rcp, table_t = false, fast_c = CK == 0 && fast_t;

#ifdef TSDF_DIAG
    int d_pairs = 0, d_valid = 0;
#endif
    for (unsigned fm = bt.n >= 32 ? fmask : fmask & ((1u << bt.n) - 1u); fm != 0; fm &= fm - 1u) {
        const Frame& fr = bt.f[__builtin_ctz(fm)];  // the frames that kept this brick, in order
#ifdef TSDF_DIAG
        ++d_pairs;
#endif
        unsigned cpx[NZ];
        double diff[NZ];
        unsigned long long okv[NZ];  // the steps' update masks
        project_part<DK, CK, NZ>(trunc, fr, px, py, pzs, pz_l, zoff, colm, nz, cpx, diff, okv);
        unsigned long long need[kH];
#pragma unroll
        for (int h = 0; h < kH; ++h) need[h] = okv[4 * h] | okv[4 * h + 1] | okv[4 * h + 2] | okv[4 * h + 3];
        if ((need[0] | need[kH - 1]) == 0) continue;
        TSDF_DDIAG(1);
#ifdef TSDF_DIAG
        ++d_valid;
#endif

        upd = true;
        if (HASH && !kHalfHash && blk < 0) {  // first frame of the batch that updates this brick: find its block
            if (HASH) {
                long long slot = 0, probe = 0;
                const unsigned long long key = pack_key(bx, by, bz);
                const long long home = ref_hash<kHalfHash>(bx, by, bz, tab.capacity, tab.int_bits);
                const int r = table_find_or_insert(tab, key, home, true, is_new, slot, probe);
                if (r < 0) {  // no space: skip the brick for the whole batch (nothing written yet);
                    if (lane == 0) {  // the host grows the table and re-runs it
                        const unsigned long long o = atomicAdd((unsigned long long*)&tab.st->n_overflow, 1ull);
                        if ((long long)o < tab.overflow_cap) tab.overflow[o] = entry;
                        atomicAdd(&s_stat[ST_OVERFLOW], 1ull);
                    }
                    return;
                }
                blk = r;
                if (is_new) {  // a fresh block starts at (1, 0, 0): nothing to load
#pragma unroll
                    for (int h = 0; h < kH; ++h) loaded[h] = ~0ull;
                }
                if (lane == 0) {
                    atomicAdd(&s_stat[ST_LOOKUPS], 1ull);
                    atomicAdd(&s_stat[ST_PROBE], (unsigned long long)probe);
                    atomicMax(&s_stat[ST_PROBE_MAX], (unsigned long long)probe);
                    if (is_new) atomicAdd(&s_stat[ST_ALLOC], 1ull);
                }
            } else {
                blk = b;
            }
        }
        // phase 4: state halves not yet in registers (the wave's first frame that needs them)
        unsigned long long ld[kH];
        unsigned long long any_ld = 0;
#pragma unroll
        for (int h = 0; h < kH; ++h) {
            ld[h] = need[h] & ~loaded[h];
            any_ld |= ld[h];
        }
        if (any_ld) {
            const size_t base = (size_t)blk * kBrickVox + (size_t)lane * kBrickEdge + zoff;
#pragma unroll
            for (int h = 0; h < kH; ++h) {
                if (!lane_in(ld[h])) continue;
                const float4 W = *(const float4*)(pool.weight + base + 4 * h);
                const float4 T = *(const float4*)(pool.tsdf + base + 4 * h);
                const float4 C = *(const float4*)(pool.color + base + 4 * h);
                ws[4 * h + 0] = W.x; ws[4 * h + 1] = W.y; ws[4 * h + 2] = W.z; ws[4 * h + 3] = W.w;
                if (canon) {  // integers >= 0 and canonical colours by construction: a range test
                    const float wm = fmaxf(fmaxf(W.x, W.y), fmaxf(W.z, W.w));
                    w_small = w_small && wm < (float)(kRcpTab - kMaxBatch - 1);
                    w_table = w_table && wm < (float)(kRcpBig - kMaxBatch - 1);
                } else {
                    w_small = w_small && small_int(W.x) && small_int(W.y) && small_int(W.z) && small_int(W.w);
                    w_table = w_table && table_int(W.x) && table_int(W.y) && table_int(W.z) && table_int(W.w);
                    c_canon = c_canon && canon_color(C.x) && canon_color(C.y) && canon_color(C.z) && canon_color(C.w);
                }
                ts[4 * h + 0] = T.x; ts[4 * h + 1] = T.y; ts[4 * h + 2] = T.z; ts[4 * h + 3] = T.w;
                if (CU) {
                    cs[4 * h + 0] = __uint_as_float((unsigned)C.x); cs[4 * h + 1] = __uint_as_float((unsigned)C.y);
                    cs[4 * h + 2] = __uint_as_float((unsigned)C.z); cs[4 * h + 3] = __uint_as_float((unsigned)C.w);
                } else {
                    cs[4 * h + 0] = C.x; cs[4 * h + 1] = C.y; cs[4 * h + 2] = C.z; cs[4 * h + 3] = C.w;
                }
            }
            // Fast paths (wave-uniform; weights grow by one per frame, so the limits leave room
            // for a whole batch): every lane's weights are small integers -> RN(1/wn) from the LDS
            // table and Markstein quotients; past the LDS part (a weight of the wave >= 4079) the
            // same from the HBM table; and, for RGB8 frames, every colour is canonical (an integer
            // B*65536+G*256+R < 2^24) -> the same for the three colour channels, in f32 with
            // RN32(1/wn) = f32(RN64(1/wn)) (checked for every table entry by the CPU tests).
            fast_t = OW1 && s_rcp && __ballot(!w_small) == 0;
            table_t = OW1 && s_rcp && !fast_t && __ballot(!w_table) == 0;
            fast_c = CK == 0 && (fast_t || table_t) && __ballot(!c_canon) == 0;
        }
#pragma unroll
        for (int h = 0; h < kH; ++h) loaded[h] |= need[h];
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            const unsigned long long m = okv[k];
            touched[k] |= m;
            nupd += (unsigned)__popcll(m);  // (wave total, scalar)
        }
        // phase 5: update in registers, straight-line; invalid steps keep their old values.
        // integrate_tsdf (grid_fusion.py:207-212): w f32 <- f64 add; f32 product; f64 average;
        // with obs_weight == 1: f32 w + 1 == f32(f64(w) + 1) exactly, and 1 * dist == dist
        // the step's new weight and colour (if it updates); a new tsdf goes into ts at once, so
        // that no quotient register crosses the branches (free space: no tsdf changes)
        float wnv[NZ], cnv[NZ];
        if (!fast_c) TSDF_DDIAG(5);
        if (fast_c) {
            // Steps in pairs (k, k+1) on the packed f32 ALU (v_pk_*: two lanes' worth per
            // instruction): w + 1, w * t, the table offset 8 * (w + 1), and the colour channels'
            // numerators and Markstein quotients.  Every value is an integer < 2^24 or the exact
            // f32 expression of the scalar form, so the results are bit-identical to it.
            // RN(1/wn) from the LDS table, or from the HBM table past its limit through a buffer
            // load (a different instruction, so the two are never merged into a flat load)
            const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void*)rcp_hbm, 0, kRcpBig * 8, kBufDword3);
            // Free space (wave-uniform): every updating voxel is at least trunc in front of the
            // surface (dist = min(1, diff / trunc) = 1 exactly) and still holds tsdf 1, so its new
            // tsdf is (w * 1 + 1) / (w + 1) = 1 exactly: the distance and tsdf quotients are skipped
            unsigned long long busy = 0;
#pragma unroll
            for (int k = 0; k < NZ; ++k)
                busy |= okv[k] & (fcmp64_mask(diff[k], trunc, kCmpOLT) | fcmp32_mask(ts[k], 1.0f, kCmpUNE));
            const bool free_space = busy == 0;
            if (free_space) TSDF_DDIAG(4);
            // the pairs' update, instantiated once for free space and once for the general case
            // (two straight-line paths: nothing of the tsdf's quotients crosses a branch)
            const auto pairs = [&](auto free_tag) {
            constexpr bool kFree = decltype(free_tag)::value;
#pragma unroll
            for (int k = 0; k < NZ; k += 2) {
                const f2 w2 = {ws[k], ws[k + 1]};
                const f2 a8 = pk_fma(w2, f2{8.0f, 8.0f}, f2{8.0f, 8.0f});  // byte offsets 8 * (w + 1)
                const unsigned o0 = (unsigned)a8.x, o1 = (unsigned)a8.y;
                double y[2];
                if (fast_t) {
                    y[0] = *(const double*)((const char*)s_rcp + o0);
                    y[1] = *(const double*)((const char*)s_rcp + o1);
                } else {
                    y[0] = __longlong_as_double((long long)__builtin_amdgcn_raw_buffer_load_b64(rt, o0, 0, 0));
                    y[1] = __longlong_as_double((long long)__builtin_amdgcn_raw_buffer_load_b64(rt, o1, 0, 0));
                }
                const f2 wn2 = w2 + 1.0f;
                f2 r2;
                if constexpr (kFree) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) r2[j] = (float)y[j];
                } else {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const double num = (double)(w2[j] * ts[k + j]) + dist_of(trunc, rtrunc, diff[k + j]);
                        const float q = (float)div_rn(num, (double)wn2[j], y[j]);
                        sel_in_place(ts[k + j], q, okv[k + j]);
                        r2[j] = (float)y[j];
                    }
                }
                // colour (grid_fusion.py:302-314): float32, round half to even; decoded by bytes
                // (v_cvt_f32_ubyte{0,1,2}), exact integer numerators by FMA, Markstein quotients;
                // the average is <= 255, so min(255, .) is a no-op
                const unsigned c0 = CU ? __float_as_uint(cs[k]) : (unsigned)cs[k];
                const unsigned c1 = CU ? __float_as_uint(cs[k + 1]) : (unsigned)cs[k + 1];
                const f2 ob = {(float)((c0 >> 16) & 0xFFu), (float)((c1 >> 16) & 0xFFu)};
                const f2 nb = {(float)((cpx[k] >> 16) & 0xFFu), (float)((cpx[k + 1] >> 16) & 0xFFu)};
                const f2 qb = div_rn32x2(pk_fma(w2, ob, nb), wn2, r2);
                const f2 og = {(float)((c0 >> 8) & 0xFFu), (float)((c1 >> 8) & 0xFFu)};
                const f2 ng = {(float)((cpx[k] >> 8) & 0xFFu), (float)((cpx[k + 1] >> 8) & 0xFFu)};
                const f2 qg = div_rn32x2(pk_fma(w2, og, ng), wn2, r2);
                const f2 orr = {(float)(c0 & 0xFFu), (float)(c1 & 0xFFu)};
                const f2 nr = {(float)(cpx[k] & 0xFFu), (float)(cpx[k + 1] & 0xFFu)};
                const f2 qr = div_rn32x2(pk_fma(w2, orr, nr), wn2, r2);
                wnv[k] = wn2.x;
                wnv[k + 1] = wn2.y;
                if (CU) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        cnv[k + j] = __uint_as_float(__builtin_amdgcn_cvt_pk_u8_f32(
                            qb[j], 2, __builtin_amdgcn_cvt_pk_u8_f32(qg[j], 1, __builtin_amdgcn_cvt_pk_u8_f32(qr[j], 0, 0u))));
                } else {
                    const f2 rb = rint2(qb), rg = rint2(qg), rr = rint2(qr);
                    const f2 cn2 = pk_fma(rb, f2{65536.0f, 65536.0f}, pk_fma(rg, f2{256.0f, 256.0f}, rr));
                    cnv[k] = cn2.x;
                    cnv[k + 1] = cn2.y;
                }
            }
            };
            if (free_space) pairs(std::true_type{});
            else pairs(std::false_type{});
        } else {
            // the exact paths: non-canonical colours or weights (table quotients where the weights
            // allow them, else IEEE divisions)
#pragma unroll
            for (int k = 0; k < NZ; ++k) {
                const float w_old = ws[k];
                const float wn = OW1 ? w_old + 1.0f : (float)((double)w_old + fr.ow);
                const double dist = dist_of(trunc, rtrunc, diff[k]);
                const double num = (double)(w_old * ts[k]) + (OW1 ? dist : fr.ow * dist);
                float q;
                if (fast_t) q = (float)div_rn(num, (double)wn, s_rcp[(int)wn]);
                else if (table_t) q = (float)div_rn(num, (double)wn, rcp_hbm[(int)wn]);
                else q = (float)(num / (double)wn);
                wnv[k] = wn;
                // colour (grid_fusion.py:302-314): float32 throughout, round half to even
                float nb, ng, nr;
                if (CK == 0) {  // packed uint8 RGB: the fold/decode round trip is exact
                    nr = (float)(cpx[k] & 0xFFu);
                    ng = (float)((cpx[k] >> 8) & 0xFFu);
                    nb = (float)((cpx[k] >> 16) & 0xFFu);
                } else {
                    const float nc = __uint_as_float(cpx[k]);
                    nb = floorf(nc / 65536.0f);
                    ng = floorf((nc - nb * 65536.0f) / 256.0f);
                    nr = nc - nb * 65536.0f - ng * 256.0f;
                }
                const float co = CU ? (float)__float_as_uint(cs[k]) : cs[k];
                const float ob = floorf(co / 65536.0f);
                const float og = floorf((co - ob * 65536.0f) / 256.0f);
                const float orr = co - ob * 65536.0f - og * 256.0f;
                const float cb = fminf(255.0f, rintf((w_old * ob + (OW1 ? nb : fr.ow32 * nb)) / wn));
                const float cg = fminf(255.0f, rintf((w_old * og + (OW1 ? ng : fr.ow32 * ng)) / wn));
                const float cr = fminf(255.0f, rintf((w_old * orr + (OW1 ? nr : fr.ow32 * nr)) / wn));
                cnv[k] = CU ? __uint_as_float((unsigned)(cb * 65536.0f + cg * 256.0f + cr))
                            : cb * 65536.0f + cg * 256.0f + cr;
                ts[k] = lane_in(okv[k]) ? q : ts[k];  // (after every read of the old ts[k])
            }
        }
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            ws[k] = lane_in(okv[k]) ? wnv[k] : ws[k];
            cs[k] = lane_in(okv[k]) ? cnv[k] : cs[k];
        }
    }
#ifdef TSDF_DIAG  // dense diagnostics in the hash-only counters: part-frame pairs computed / valid
    if (!HASH && lane == 0) {
        atomicAdd(&s_stat[ST_PROBE], (unsigned long long)d_pairs);
        atomicAdd(&s_stat[ST_LOOKUPS], (unsigned long long)d_valid);
    }
#endif
    if constexpr (kHalfHash) {
        unsigned long long any = 0;
#pragma unroll
        for (int k = 0; k < NZ; ++k) any |= touched[k];
        if (any == 0) return;  // this half updated nothing
    } else if (!upd) {
        return;  // no frame of the batch updated this brick
    }

#pragma unroll
    for (int k = 0; k < NZ; ++k) nuniq += (unsigned)__popcll(touched[k]);
    // phase 6: store the changed halves once (a new hash block is written whole: its init)
    const size_t base = (size_t)blk * kBrickVox + (size_t)lane * kBrickEdge + zoff;
#pragma unroll
    for (int h = 0; h < kH; ++h) {
        if (!lane_in(loaded[h])) continue;
        *(float4*)(pool.weight + base + 4 * h) = make_float4(ws[4 * h], ws[4 * h + 1], ws[4 * h + 2], ws[4 * h + 3]);
        *(float4*)(pool.tsdf + base + 4 * h) = make_float4(ts[4 * h], ts[4 * h + 1], ts[4 * h + 2], ts[4 * h + 3]);
        if (CU)
            *(float4*)(pool.color + base + 4 * h) =
                make_float4((float)__float_as_uint(cs[4 * h]), (float)__float_as_uint(cs[4 * h + 1]),
                            (float)__float_as_uint(cs[4 * h + 2]), (float)__float_as_uint(cs[4 * h + 3]));
        else
            *(float4*)(pool.color + base + 4 * h) = make_float4(cs[4 * h], cs[4 * h + 1], cs[4 * h + 2], cs[4 * h + 3]);
    }
    if constexpr (HASH) {  // voxel-entry bits: word z, bit (x*8+y); this wave owns words zoff .. zoff+NZ-1
        unsigned long long mine = 0;
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            if (lane == k) mine = touched[k];
        }
        if (lane < NZ) {
            unsigned long long* o = tab.occ + (size_t)blk * kBrickEdge + zoff + lane;
            if (is_new) coh_store(o, mine);
            else if (mine) atomicOr(o, mine);
        }
    }
    if (lane == 0) atomicAdd(&s_stat[ST_TOUCHED], 1ull);
}

__device__ inline void flush_stats(unsigned long long* s_stat, unsigned long long* stats) {
    const int tid = threadIdx.x;
    if (tid < kNStat && s_stat[tid]) {
        unsigned long long* dst = stats + tid * kStatSpread + (blockIdx.x & (kStatSpread - 1));
        if (tid == ST_PROBE_MAX) atomicMax(dst, s_stat[tid]);
        else atomicAdd(dst, s_stat[tid]);
    }
}

// Conservative cull of every brick (one lane each) against every frame of the batch, and
// compaction of the bricks seen by at least one frame into a list of (brick | frame mask << 24):
// wave ballot + LDS prefix over the 4 waves + ONE atomicAdd per workgroup.
constexpr int kCullWG = 512;  // k_cull: 8 waves, wave w culls frames w and w + 8

// Wave-level append of the kept bricks (lane: brick e, its frame mask) to the sub-list of their cost
// class (frames kept): one atomicAdd per class with survivors.
// The fused hash launch's cull also finds or inserts every kept brick's block (one lane per brick, a
// linear probe of the power-of-two table: about one slot at the bench's load factors; a new block
// from the pool, its key by CAS into the first tombstone or empty slot of the probe) and leaves it
// in the brick's claim word for the integrate of the next launch (integrate_brick).  Nothing else
// inserts during a fused launch (its integrate only reads blocks its cull found a launch earlier),
// and the bricks of a batch are distinct, so a lost CAS is another brick's key: the probe goes on.
// The cull's wave then initialises its new blocks -- (1, 0, 0) and no entries, 64 lanes per block --
// and records them for k_free_unused (a block the batch leaves without an entry is freed at the end
// of the call).  kResFail: the pool or table is full (the brick goes to the host's exact re-run).
#ifndef TSDF_CULL_PROBE8  // cull_find_or_insert walks the table 8 slots per dependent load (round 6)
#define TSDF_CULL_PROBE8 1  // instead of one (0: round 5's lane-serial probe, for A/B)
#endif
// A block taken from the pool for a key whose probe then ended without inserting it (the table ran
// out of slots after a lost race): recorded in the inserted list as -2 - block, so k_free_unused
// returns it to the free list at the end of the call (round-5 advisor: it stayed counted as used).
__device__ inline void spare_block(const Table& t, int blk) {
    if (blk < 0) return;
    const unsigned long long k = atomicAdd((unsigned long long*)&t.st->n_inserted, 1ull);
    if ((long long)k < t.ins_cap) t.ins_list[k] = -2 - blk;
}
__device__ inline void cull_probe_stats(unsigned long long* s_stat, long long n, bool alloc) {
    if (alloc) atomicAdd(&s_stat[ST_ALLOC], 1ull);
    atomicAdd(&s_stat[ST_LOOKUPS], 1ull);
    atomicAdd(&s_stat[ST_PROBE], (unsigned long long)n);
    atomicMax(&s_stat[ST_PROBE_MAX], (unsigned long long)n);
}
__device__ inline int cull_find_or_insert(const Vol& v, const Table& t, unsigned e, unsigned long long* s_stat,
                                          bool& fresh) {
    fresh = false;
    const int nb12 = v.nb[1] * v.nb[2];
    const int bx = (int)e / nb12, r = (int)e - bx * nb12, by = r / v.nb[2], bz = r - by * v.nb[2];
    const unsigned long long key = pack_key(bx, by, bz);
    // the table's fields once, into registers (t may be read through an opaque pointer: opaque)
    unsigned long long* const keys = t.keys;
    int* const vals = t.vals;
    const long long cap = t.capacity, max_blocks = t.max_blocks;
    const long long mask = cap - 1;
    long long s = ref_hash<true>(bx, by, bz, cap, t.int_bits);
    long long tomb = -1, tomb_n = 0;
    int blk = -1;
#if TSDF_CULL_PROBE8
    if (cap >= 8) {
        // Eight slots per step: the aligned 64-B group of keys holding slot s (four 16-B loads) and
        // its 32 B of slot values, issued together -- one memory latency per 8 slots instead of one
        // per slot, so a lane's chain at a high load factor is an eighth as long (the wave waits for
        // its longest).  Plain loads: in this launch a key only ever goes from empty / tombstone to
        // a key (no removal runs beside the cull), and this brick's key is inserted by no one but
        // this lane, so a stale read can only show an empty / tombstone slot that another brick has
        // just taken -- its CAS then fails and the probe goes on, as on a lost race; a key from an
        // earlier launch (and its value) is visible from the launch's start.
        for (long long n = 0; n < cap;) {
            const long long g0 = s & ~7ll;
            const int off = (int)(s - g0);
            unsigned long long kk[8];
            int vv[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const ulonglong2 q = *(const ulonglong2*)(keys + g0 + 2 * j);
                kk[2 * j] = q.x;
                kk[2 * j + 1] = q.y;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int4 q = *(const int4*)(vals + g0 + 4 * j);
                vv[4 * j] = q.x, vv[4 * j + 1] = q.y, vv[4 * j + 2] = q.z, vv[4 * j + 3] = q.w;
            }
            unsigned hit = 0, emp = 0, tm = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                hit |= (unsigned)(kk[i] == key) << i;
                emp |= (unsigned)(kk[i] == kEmpty) << i;
                tm |= (unsigned)(kk[i] == kTomb) << i;
            }
            const unsigned from = 0xFFu << off;  // the slots at or after s
            const unsigned stop = (hit | emp) & from;
            const int i = stop ? __builtin_ctz(stop) : 8;  // the first key match or empty slot
            const unsigned before = tm & from & ((1u << i) - 1u);  // tombstones before it
            if (tomb < 0 && before) {
                tomb = g0 + __builtin_ctz(before);
                tomb_n = n + (__builtin_ctz(before) - off);
            }
            if (i == 8) {  // no stop in the group: on to the next
                n += 8 - off;
                s = (g0 + 8) & mask;
                continue;
            }
            long long vi = 0;  // vv[i] without a dynamically indexed register array
#pragma unroll
            for (int j = 0; j < 8; ++j) vi = j == i ? vv[j] : vi;
            if ((hit >> i) & 1u) {
                cull_probe_stats(s_stat, n + (i - off), false);
                spare_block(t, blk);  // (never holds one: only this lane inserts this key)
                return (vi >= 0 && vi < max_blocks) ? (int)vi : kResFail;  // (a found key's value is always set)
            }
            // absent: a block from the pool (kept across lost races), then the key by CAS into the
            // first tombstone of the probe, else this empty slot
            const long long target = tomb >= 0 ? tomb : g0 + i;
            const long long tn = tomb >= 0 ? tomb_n : n + (i - off);
            const unsigned long long expect = tomb >= 0 ? kTomb : kEmpty;
            if (blk < 0) blk = pool_alloc(t);
            if (blk < 0) return kResFail;  // pool exhausted
            if (atomicCAS(&keys[target], expect, key) == expect) {
                coh_store(&vals[target], blk);
                const unsigned long long k = atomicAdd((unsigned long long*)&t.st->n_inserted, 1ull);
                if ((long long)k < t.ins_cap) t.ins_list[k] = (int)e;
                cull_probe_stats(s_stat, tn, true);
                fresh = true;
                return blk;
            }
            // another brick's key took the slot: probe on just past it
            n = tn + 1;
            s = (target + 1) & mask;
            tomb = -1;
        }
        spare_block(t, blk);
        return kResFail;  // table full (the growth policy keeps it below 31/32)
    }
#endif
    for (long long n = 0; n < cap; ++n) {  // one slot per step (tables of < 8 slots; A/B)
        const unsigned long long k = coh_load(&keys[s]);
        if (k == key) {
            const int b = coh_load(&vals[s]);
            cull_probe_stats(s_stat, n, false);
            spare_block(t, blk);
            return (b >= 0 && b < max_blocks) ? b : kResFail;  // (a found key's value is always set)
        }
        if (k == kTomb) {
            if (tomb < 0) tomb = s;
        } else if (k == kEmpty) {  // absent: insert at the first tombstone of the probe, else here
            const long long target = tomb >= 0 ? tomb : s;
            const unsigned long long expect = tomb >= 0 ? kTomb : kEmpty;
            if (blk < 0) blk = pool_alloc(t);
            if (blk < 0) return kResFail;  // pool exhausted
            if (atomicCAS(&keys[target], expect, key) == expect) {
                coh_store(&vals[target], blk);
                const unsigned long long i = atomicAdd((unsigned long long*)&t.st->n_inserted, 1ull);
                if ((long long)i < t.ins_cap) t.ins_list[i] = (int)e;
                cull_probe_stats(s_stat, n, true);
                fresh = true;
                return blk;
            }
            s = target;  // another brick's key took the slot: probe on from it
            tomb = -1;
            continue;
        }
        s = (s + 1) & mask;
    }
    spare_block(t, blk);
    return kResFail;  // table full (the growth policy keeps it below 31/32)
}

template <bool HASH>
__device__ inline void append_kept(const Vol& v, ListEntry* list, unsigned int* count, unsigned long long* s_stat,
                                   int* res, unsigned e, unsigned fmask, int ncls, const Table* tab = nullptr,
                                   const Pool* pool = nullptr) {
    // ncls: the batch's frames (cost classes 1..ncls; wave-uniform)
    const int lane = lane_id();
    const int cls = __popc(fmask);
    const unsigned long long any = __ballot(cls != 0);
    if (!any) return;
    unsigned n_cls = 0, rank = 0;
    for (int c = 1; c <= ncls; ++c) {
        const unsigned long long m = __ballot(cls == c);
        if (lane == c) n_cls = (unsigned)__popcll(m);
        if (cls == c) rank = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
    }
    unsigned base = 0;  // lanes 1..8 reserve their class's slots at once
    if (lane >= 1 && lane <= ncls && n_cls) base = atomicAdd(&count[lane], n_cls);
    if (lane == 0) atomicAdd(&s_stat[ST_VISITED], (unsigned long long)__popcll(any));
    base = __shfl(base, cls);
    const unsigned nbk = (unsigned)(v.nb[0] * v.nb[1] * v.nb[2]);
    bool fresh = false;
    int blk = kResFree;
    if (cls && base + rank < nbk) {
        list[(size_t)(cls - 1) * nbk + base + rank] = (ListEntry)e | ((ListEntry)fmask << 32);
        // the brick's claim word for this batch: its block (found or inserted), or kResFail
        if (HASH && res) res[e] = blk = tab ? cull_find_or_insert(v, *tab, e, s_stat, fresh) : kResFree;
    }
    if (HASH && res && pool) {  // new blocks start at (1, 0, 0) with no entries: 64 lanes per block
        for (unsigned long long m = __ballot(fresh); m; m &= m - 1) {
            const int b = __shfl(blk, __ffsll((long long)m) - 1);
            const size_t o = (size_t)b * kBrickVox + (size_t)lane * kBrickEdge;
            const float4 one = make_float4(1.0f, 1.0f, 1.0f, 1.0f), zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            *(float4*)(pool->tsdf + o) = one;
            *(float4*)(pool->tsdf + o + 4) = one;
            *(float4*)(pool->weight + o) = zero;
            *(float4*)(pool->weight + o + 4) = zero;
            *(float4*)(pool->color + o) = zero;
            *(float4*)(pool->color + o + 4) = zero;
            if (lane < kBrickEdge) coh_store(tab->occ + (size_t)b * kBrickEdge + lane, 0ull);
        }
    }
}

// Brick culling for one batch: one workgroup per G superbricks (64 bricks each, Vol::sb), one wave
// per (superbrick, frame) pair at a time, each lane testing its brick against the frame; the
// per-brick frame masks meet in LDS and wave g appends superbrick g's kept bricks to the list (one
// atomicAdd per cost class with survivors).  A test is one cull_brick deep; a wave takes
// ceil(G * frames / waves) pairs in turn.  (Round 3 dropped the superbrick-level test that ran
// first: an invisible brick leaves cull_brick at its bounding-sphere test anyway, and a visible
// superbrick cost two test latencies instead of one -- +2.7 % dense, +2.6 % on an eighth shard.)  G > 1 (fused launches over large volumes,
// Base::cull_per_wg): the test is latency-bound, so a workgroup's fixed costs (start, barriers,
// list atomics, statistics) are shared by G superbricks and the stage takes fewer of the CUs'
// slots while the integrate still runs (+1.8 % at 512^3); on small shards the cull runs in the
// launch's tail, where its latency counts, and G = 1.
constexpr int kCullGMax = 4;
template <bool HASH, bool P2 = false>
__device__ inline void cull_superbrick(const Vol& v, const Batch& bt, const Table& tab, ListEntry* list,
                                       unsigned int* count, unsigned long long* stats, int wgi,
                                       unsigned* s_mask, unsigned long long* s_stat, int* res = nullptr,
                                       int G = 1, const Pool* pool = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), n_waves = (int)(blockDim.x >> 6);
    if (tid < 64 * G) s_mask[tid] = 0u;
    if (tid < kNStat) s_stat[tid] = 0;
    __syncthreads();
    const int nsx = (v.nb[0] + (1 << v.sb[0]) - 1) >> v.sb[0];
    const int nsy = (v.nb[1] + (1 << v.sb[1]) - 1) >> v.sb[1];
    const int nsz = (v.nb[2] + (1 << v.sb[2]) - 1) >> v.sb[2];
    const int n_sb = nsx * nsy * nsz;
    const int ex = 1 << v.sb[0], ey = 1 << v.sb[1], ez = 1 << v.sb[2];
    const int lz = lane & (ez - 1), ly = (lane >> v.sb[2]) & (ey - 1), lx = lane >> (v.sb[1] + v.sb[2]);
    for (int p = wave; p < G * bt.n; p += n_waves) {  // (superbrick g, frame f) pairs
        const int g = p / bt.n, f = p - g * bt.n;
        const int si = wgi * G + g;
        if (si >= n_sb) continue;
        const int sx = si / (nsy * nsz), sr = si - sx * (nsy * nsz), sy = sr / nsz, sz = sr - sy * nsz;
        const int bx = sx * ex + lx, by = sy * ey + ly, bz = sz * ez + lz;
        const Frame& fr = bt.f[f];
        bool test = bx < v.nb[0] && by < v.nb[1] && bz < v.nb[2];
        if (HASH && v.n_shards > 1 && test) {  // bucket-range ownership (shards use cull_owned)
            const long long home = ref_hash<P2>(bx, by, bz, tab.shard_cap, tab.int_bits);
            test = shard_of<P2>(home, v.n_shards, tab.shard_cap) == v.shard;
        }
        if (test && cull_brick(v, fr, bt.pg, brick_box(v, fr.eye, bx, by, bz))) atomicOr(&s_mask[g * 64 + lane], 1u << f);
    }
    __syncthreads();
    const int si = wgi * G + wave;
    if (wave < G && si < n_sb) {  // append the kept bricks to the sub-list of their cost class (frames kept)
        const int sx = si / (nsy * nsz), sr = si - sx * (nsy * nsz), sy = sr / nsz, sz = sr - sy * nsz;
        const int bx = sx * ex + lx, by = sy * ey + ly, bz = sz * ez + lz;
        append_kept<HASH>(v, list, count, s_stat, res, (unsigned)(((long long)bx * v.nb[1] + by) * v.nb[2] + bz),
                          s_mask[wave * 64 + lane], bt.n, P2 ? &tab : nullptr, pool);
    }
    __syncthreads();
    flush_stats(s_stat, stats);
}

// The cull of a bucket-range hash shard (Table::owned): its bricks are spread over the whole
// extent (one in n_shards, by home bucket), so instead of walking every superbrick of the extent it
// walks only the bricks the shard owns, 64 per workgroup (lane = brick, one wave per frame at a
// time: one brick test deep, no superbrick level).  An eighth shard culls an eighth of the bricks.
template <bool HASH>
__device__ inline void cull_owned(const Vol& v, const Batch& bt, const Table& tab, ListEntry* list,
                                  unsigned int* count, unsigned long long* stats, int wgi, unsigned* s_mask,
                                  unsigned long long* s_stat, int* res, const Pool* pool = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), n_waves = (int)(blockDim.x >> 6);
    if (tid < 64) s_mask[tid] = 0u;
    if (tid < kNStat) s_stat[tid] = 0;
    __syncthreads();
    const int i = wgi * 64 + lane;
    const bool have = i < tab.n_owned;
    const int e = have ? tab.owned[i] : 0;
    const int nb12 = v.nb[1] * v.nb[2];
    const int bx = e / nb12, r = e - bx * nb12, by = r / v.nb[2], bz = r - by * v.nb[2];
    for (int f = wave; f < bt.n; f += n_waves) {
        const Frame& fr = bt.f[f];
        if (have && cull_brick(v, fr, bt.pg, brick_box(v, fr.eye, bx, by, bz))) atomicOr(&s_mask[lane], 1u << f);
    }
    __syncthreads();
    if (wave == 0) append_kept<HASH>(v, list, count, s_stat, res, (unsigned)e, have ? s_mask[lane] : 0u, bt.n, &tab, pool);
    __syncthreads();
    flush_stats(s_stat, stats);
}

template <bool HASH>
__global__ __launch_bounds__(kCullWG) void k_cull(Vol v, Batch bt, Table tab, ListEntry* list,
                                                  unsigned int* count, unsigned long long* stats) {
    __shared__ unsigned s_mask[64];
    __shared__ unsigned long long s_stat[kNStat];
    if (HASH && tab.owned) cull_owned<HASH>(v, bt, tab, list, count, stats, blockIdx.x, s_mask, s_stat, nullptr);
    else cull_superbrick<HASH>(v, bt, tab, list, count, stats, blockIdx.x, s_mask, s_stat);
}

// Integrate the listed bricks: each wave takes list entries gw, gw + NW, ... (NW = waves in the
// grid, all resident), so the work is spread evenly whatever the frames see.  `count` (device)
// gives the list length written by k_cull; with count == nullptr the first n_list entries are
// used (hash overflow re-run).
#ifndef TSDF_PRIO  // progress priority of the dense integrate's waves (integrate_items)
#define TSDF_PRIO 1
#endif
#ifndef TSDF_PRIO_HASH  // ... and of the hash integrate's
#define TSDF_PRIO_HASH 1
#endif
#ifndef TSDF_PRIO_MIN  // ... for workgroups with at least this many list items (brick parts)
#define TSDF_PRIO_MIN 64
#endif
#ifndef TSDF_PRIO_MIN_HASH  // ... the hash integrate's
#define TSDF_PRIO_MIN_HASH 16
#endif
// A pointer the compiler cannot see through: loads from it are neither merged with loads before
// it nor speculated out of the conditional blocks that use them.  The fused launches read their
// volume geometry, pool and (hash) table fields through such pointers to their own kernarg copy,
// so those loads stay where the fields are used (scalar loads, scalar-cache hits) instead of being
// hoisted to the kernel's entry and held in scalar registers across the item and frame loops,
// where the frame constants and step masks need them: with them held, SGPRs spilled to VGPR lanes
// (v_writelane / v_readlane, VALU instructions) and, in the hash launch, VGPRs to scratch.
template <typename T>
__device__ inline const __attribute__((address_space(4))) T* opaque(const __attribute__((address_space(4))) T* p) {
    asm volatile("" : "+s"(p));
    return p;
}

typedef const __attribute__((address_space(4))) Vol* VolP;
// The volume of an item: re-read per item through an opaque pointer (v must be the launch's kernarg
// copy), so its fields are not hoisted out of the item loop and held across it.
__device__ inline const Vol& item_vol(const Vol& v) { return *(const Vol*)opaque((VolP)&v); }

template <bool HASH, int DK, int CK, bool OW1, int NZ, bool CU>
__device__ inline void integrate_items(const Vol& v, const Batch& bt, const Pool& pool, const Table& tab,
                                       const ListEntry* list, unsigned int* count, int n_list, int wave,
                                       int n_waves, unsigned long long* s_stat, const double* s_rcp,
                                       unsigned* s_next, int wg, int n_wg, int* res, unsigned& nupd,
                                       unsigned& nuniq);
template <bool HASH, int DK, int CK, bool OW1, int NZ, bool CU = false>
__device__ inline void integrate_list(const Vol& v, const Batch& bt, const Pool& pool, const Table& tab,
                                      const ListEntry* list, unsigned int* count, int n_list, int wave,
                                      int n_waves, unsigned long long* s_stat, const double* s_rcp,
                                      unsigned* s_next = nullptr, int wg = 0, int n_wg = 1, int* res = nullptr) {
    wave = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the list walk stays scalar
    unsigned nupd = 0, nuniq = 0;  // the wave's voxel updates over all its items (ST_VOXELS, ST_UNIQUE; wave-uniform)
    integrate_items<HASH, DK, CK, OW1, NZ, CU>(v, bt, pool, tab, list, count, n_list, wave, n_waves, s_stat, s_rcp,
                                           s_next, wg, n_wg, res, nupd, nuniq);
    if (lane_id() == 0 && nupd) {
        atomicAdd(&s_stat[ST_VOXELS], (unsigned long long)nupd);
        atomicAdd(&s_stat[ST_UNIQUE], (unsigned long long)nuniq);
    }
}

template <bool HASH, int DK, int CK, bool OW1, int NZ, bool CU>
__device__ inline void integrate_items(const Vol& v, const Batch& bt, const Pool& pool, const Table& tab,
                                       const ListEntry* list, unsigned int* count, int n_list, int wave,
                                       int n_waves, unsigned long long* s_stat, const double* s_rcp,
                                       unsigned* s_next, int wg, int n_wg, int* res, unsigned& nupd,
                                       unsigned& nuniq) {
    constexpr int parts = 8 / NZ;  // waves per listed brick
    if (!count) {  // a flat list of n_list entries (hash overflow re-run)
        for (int e = wave; e < n_list * parts; e += n_waves)
            integrate_brick<HASH, DK, CK, OW1, NZ, CU>(item_vol(v), bt, pool, tab, list[e / parts], (e % parts) * NZ,
                                                   s_stat, s_rcp, nupd, nuniq);
        return;
    }
    // k_cull's list: one sub-list per cost class (frames kept, 1..kMaxBatch), taken most frames
    // first, so that the round-robin hands every wave a similar amount of work (the longest-job-
    // first order of list scheduling)
    const unsigned nbk = (unsigned)(v.nb[0] * v.nb[1] * v.nb[2]);
    // (cost classes 1..bt.n: the batch's frames)
    const int ncls = __builtin_amdgcn_readfirstlane(bt.n);
    int total = 0;
    for (int c = 0; c < ncls; ++c) total += (int)min(coh_load(&count[c + 1]), nbk);
    int c = ncls - 1;
    unsigned k0 = 0;  // list ordinal where class c starts (classes visited in descending order)
    // the length of class c only (one scalar live across the items; the next class's is read when
    // the walk reaches it -- at most kMaxBatch - 1 times per wave)
    unsigned nc = min(coh_load(&count[c + 1]), nbk);
    if (s_next) {
        // Items dealt round-robin to workgroups (still longest first) and taken dynamically by
        // the workgroup's waves from an LDS counter: a wave that
        // drew short items takes more, so a workgroup ends when its last item does, not when its
        // unluckiest wave's static share does (the tail of small shards: few items per wave).
        // Progress priority (hash launches): the SIMDs arbitrate VALU issue by priority, then age,
        // so of the workgroups sharing a CU the first-dispatched one runs ahead and the last runs
        // its tail alone.  A wave's priority falls as its workgroup's share is taken (3 below 1/2,
        // 2 below 13/16, 1 below 15/16, then 0), so a workgroup that lags keeps the issue slots
        // until it has caught up.  Hash: +4 % on one GPU (z-half waves that wait for their
        // partner's claim word stop losing the SIMD to older workgroups), and with 768-thread
        // workgroups +5 % on an eighth shard too (~35 items per workgroup; TSDF_PRIO_MIN_HASH 16).
        // Dense: -2.9 % time per 16-frame launch on one GPU, but +3 % on an eighth shard, so from
        // 64 items per workgroup (profiles/r04_p/).
        constexpr bool kPrio = HASH ? TSDF_PRIO_HASH != 0 : TSDF_PRIO != 0;
#if TSDF_XCD_DEAL
        // XCD-aware dealing: the launch's workgroups go to the 8 XCDs round-robin (workgroup w on
        // XCD (w + r) % 8, the rotation r carried over from the dispatches before: measured from
        // the workgroups' XCC_ID registers, profiles/r05_shards/), so dealing brick k to workgroup
        // k mod n_wg would hand each XCD every 8th
        // brick of the list, spread over the whole image.  Renumbered, workgroup w deals as
        // (w % 8) * n_wg/8 + w / 8: each XCD takes runs of n_wg/8 consecutive bricks (neighbours
        // in the cull's order), whose gathers share its L2.
        if ((n_wg & 7) == 0) wg = (wg & 7) * (n_wg >> 3) + (wg >> 3);
#endif
        const unsigned mine = total > wg ? (unsigned)((total - wg + n_wg - 1) / n_wg) * parts : 0u;
        const bool use_prio = kPrio && mine >= (HASH ? TSDF_PRIO_MIN_HASH : TSDF_PRIO_MIN);  // (wave-uniform)
        [[maybe_unused]] int prio = 3;
        if (use_prio) __builtin_amdgcn_s_setprio(3);
        // (TSDF_ITEM_PREFETCH: each wave takes its next item, and issues the load of its list
        // entry, before it integrates the current one -- one item held in reserve per wave)
        const auto take = [&](ListEntry& e, int& zoff) -> bool {
            unsigned j = 0;
            if (lane_id() == 0) j = atomicAdd(s_next, 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            if (use_prio) {
                const unsigned q = j * 16u;
                const int p = q < mine * 8u ? 3 : q < mine * 13u ? 2 : q < mine * 15u ? 1 : 0;
                if (p != prio) {
                    prio = p;
                    if (p == 2) __builtin_amdgcn_s_setprio(2);
                    else if (p == 1) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(0);
                }
            }
            // bricks dealt to workgroups (brick k to workgroup k mod n_wg), the parts of one brick
            // taken one after the other, so they run side by side on the workgroup's waves and
            // share their depth / colour gathers in the CU's cache
            const long long k = (long long)wg + (long long)(j / parts) * n_wg;  // increasing for this wave
            if (k >= (long long)total) return false;
            while (c > 0 && (unsigned)k - k0 >= nc) {
                k0 += nc;
                --c;
                nc = min(coh_load(&count[c + 1]), nbk);
            }
            e = list[(size_t)c * nbk + ((unsigned)k - k0)];
            zoff = (int)(j % parts) * NZ;
            return true;
        };
        ListEntry e = 0;
        int zoff = 0;
#if TSDF_ITEM_PREFETCH
        bool have = take(e, zoff);
        while (have) {
            ListEntry en = 0;
            int zn = 0;
            const bool more = take(en, zn);
            // (the parts of a brick stay in one workgroup: the hash's z-halves meet in res)
            integrate_brick<HASH, DK, CK, OW1, NZ, CU>(item_vol(v), bt, pool, tab, e, zoff, s_stat, s_rcp, nupd, nuniq, res);
            have = more;
            e = en;
            zoff = zn;
        }
#else
        while (take(e, zoff))  // (the parts of a brick stay in one workgroup: the hash's z-halves meet in res)
            integrate_brick<HASH, DK, CK, OW1, NZ, CU>(item_vol(v), bt, pool, tab, e, zoff, s_stat, s_rcp, nupd, nuniq, res);
#endif
        if (use_prio) __builtin_amdgcn_s_setprio(0);
        return;
    }
    for (int e = wave; e < total * parts; e += n_waves) {
        const unsigned k = (unsigned)(e / parts);
        while (c > 0 && k - k0 >= nc) {
            k0 += nc;
            --c;
            nc = min(coh_load(&count[c + 1]), nbk);
        }
        integrate_brick<HASH, DK, CK, OW1, NZ, CU>(item_vol(v), bt, pool, tab, list[(size_t)c * nbk + (k - k0)],
                                               (e % parts) * NZ, s_stat, s_rcp, nupd, nuniq, res);
    }
}

// Occupancy targets (waves per SIMD) of the integrate kernels.  Dense k_fused: 6 (<= 80 VGPRs;
// 512-thread workgroups, 3 per CU, 99 KB of LDS) -- measured 8 % faster than 4 at 512^3
// (DESIGN.md §4); 8 would spill to scratch.  Hash (NZ = 8, the probe state) and in-line: 4.
#ifndef TSDF_DENSE_WAVES
#define TSDF_DENSE_WAVES 6
#endif
#ifndef TSDF_HASH_WAVES
#define TSDF_HASH_WAVES 4
#endif
template <bool HASH, int DK, int CK, bool OW1, int NZ = 8>
// (the in-line k_integrate: 256-thread workgroups with a 32 KB LDS table fit 4 per CU, so 4 waves
// per SIMD whatever the registers allow)
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(TSDF_HASH_WAVES))) void k_integrate(Vol v, Batch bt, Pool pool, Table tab,
                                                  unsigned long long* stats, const ListEntry* list,
                                                  unsigned int* count, int n_list) {
    (void)v;  // read through its kernarg copy (the first parameter: offset 0), see item_vol
    const Vol& vk = *(const Vol*)opaque((VolP)__builtin_amdgcn_kernarg_segment_ptr());
    __shared__ unsigned long long s_stat[kNStat];
    __shared__ double s_rcp[OW1 ? kRcpTab : 1];  // RN(1/n): weights are small integers when ow == 1
    __shared__ unsigned s_next;                  // the workgroup's next list item (integrate_list)
    const int tid = threadIdx.x;
    if (tid < kNStat) s_stat[tid] = 0;
    if (tid == 0) s_next = 0;
    if (OW1)  // 32 KB table copied with 16-byte loads (computing it cost 16 f64 divisions per thread)
        for (int i = tid; i < kRcpTab / 2; i += kWG) ((double2*)s_rcp)[i] = ((const double2*)vk.rcp)[i];
    __syncthreads();
    integrate_list<HASH, DK, CK, OW1, NZ>(vk, bt, pool, tab, list, count, n_list,
                                          blockIdx.x * (kWG / 64) + (tid >> 6), gridDim.x * (kWG / 64),
                                          s_stat, OW1 ? s_rcp : nullptr, &s_next, blockIdx.x, gridDim.x);
    __syncthreads();
    flush_stats(s_stat, stats);
}

// Per frame, before the cull (one pass over the image): the packed RGB8 image, the max-depth
// pyramid levels 1..6
// (texel = max over a 2^L x 2^L block, metres, 0 for invalid/outside) and the reset of the
// brick-list counter.  One 1024-thread workgroup per 64x64 tile, 2x2 pixels per thread.
template <int REDUCE>
__device__ inline void pyr_level(const PyrGeo& pg, float* pyr, int L, const float (*src)[33],
                                 float (*dst)[33], int n, int tx = blockIdx.x, int ty = blockIdx.y) {
    const int t = threadIdx.x;
    if (t < n * n) {
        const int rr = t / n, cc = t - rr * n;
        const float m = fmaxf(fmaxf(src[2 * rr][2 * cc], src[2 * rr][2 * cc + 1]),
                              fmaxf(src[2 * rr + 1][2 * cc], src[2 * rr + 1][2 * cc + 1]));
        dst[rr][cc] = m;
        const int X = tx * n + cc, Y = ty * n + rr;
        if (X < pg.w[L] && Y < pg.h[L]) pyr[pg.off[L] + Y * pg.w[L] + X] = m;
    }
}

// k_prep for u16 (DK = 0) or f64 (DK = 1) depth + RGB8 with W % 4 == 0 and aligned buffers (the
// common case): 512 threads per 64x64 tile, 4x2 pixels per thread, moved with 8-byte u16 depth
// loads (two 16-byte loads for f64), three 4-byte colour loads per row (4 packed RGB pixels) and
// one 16-byte RGBX store per row -- instead of one 2-byte and three 1-byte loads and one 4-byte
// store per pixel.  Same outputs as k_prep<DK, 0>.
template <int DK = 0>
__device__ inline void prep_vec_tile(const Batch& bt, unsigned int* count, int tx, int ty, int tf,
                                     float (*sa)[33], float (*sb)[33]) {
    const Frame& fr = bt.f[tf];
    float* pyr = (float*)fr.pyr;
    const int t = threadIdx.x, r = t >> 4, c = t & 15;
    if (count && t < kCountWords && tx == 0 && ty == 0 && tf == 0) coh_store(count + t, 0u);  // list counters
    const bool act = t < 512;  // (a fused launch's workgroup may be larger: the rest only meets the barriers)
    const int x0 = tx * 64 + c * 4, y0 = ty * 64 + r * 2;
    float ma = 0.0f, mb = 0.0f;  // level-1 texels (x0/2, y0/2) and (x0/2 + 1, y0/2)
    if (act && x0 < fr.W) {
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int y = y0 + dy;
            if (y >= fr.H) continue;
            const size_t p = (size_t)y * fr.W + x0;
            uint2 dd = make_uint2(0u, 0u);  // (u16: the 4 pixels' depth, masked)
            if (DK == 1) {  // f64 metres (the reference's own depth_im)
                const double2 d0 = *(const double2*)((const double*)fr.depth_src + p);
                const double2 d1 = *(const double2*)((const double*)fr.depth_src + p + 2);
                ma = fmaxf(ma, fmaxf((float)d0.x, (float)d0.y));
                mb = fmaxf(mb, fmaxf((float)d1.x, (float)d1.y));
            } else {
                dd = *(const uint2*)((const unsigned short*)fr.depth_src + p);
                if (fr.depth_mask) {  // the demos' depth_im[depth_im == 65.535] = 0
                    unsigned lo0 = dd.x & 0xFFFFu, hi0 = dd.x >> 16, lo1 = dd.y & 0xFFFFu, hi1 = dd.y >> 16;
                    lo0 = lo0 == 65535u ? 0u : lo0;
                    hi0 = hi0 == 65535u ? 0u : hi0;
                    lo1 = lo1 == 65535u ? 0u : lo1;
                    hi1 = hi1 == 65535u ? 0u : hi1;
                    dd = make_uint2(lo0 | (hi0 << 16), lo1 | (hi1 << 16));
                    *(uint2*)(fr.depth_mask + p) = dd;
                }
                ma = fmaxf(ma, fmaxf((float)(dd.x & 0xFFFFu) * 1e-3f, (float)(dd.x >> 16) * 1e-3f));
                mb = fmaxf(mb, fmaxf((float)(dd.y & 0xFFFFu) * 1e-3f, (float)(dd.y >> 16) * 1e-3f));
            }
            if (fr.rgbx) {  // (frames the integrate cannot gather in place, frame_bufs)
                const unsigned* q = (const unsigned*)((const unsigned char*)fr.color + 3 * p);
                const unsigned a = q[0], b = q[1], cc = q[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
                const uint4 c4 = make_uint4(a & 0xFFFFFFu, (a >> 24) | ((b & 0xFFFFu) << 8),
                                            (b >> 16) | ((cc & 0xFFu) << 16), cc >> 8);
                if (DK == 2) {  // 8-byte texels (depth, colour)
                    uint4* t = (uint4*)((uint2*)fr.rgbx + p);
                    t[0] = make_uint4(dd.x & 0xFFFFu, c4.x, dd.x >> 16, c4.y);
                    t[1] = make_uint4(dd.y & 0xFFFFu, c4.z, dd.y >> 16, c4.w);
                } else {
                    *(uint4*)((unsigned*)fr.rgbx + p) = c4;
                }
            }
        }
    }
    const PyrGeo& pg = bt.pg;
    const auto put = [&](int L, int X, int Y, float m) {
        if (X < pg.w[L] && Y < pg.h[L]) pyr[pg.off[L] + Y * pg.w[L] + X] = m;
    };
    if (act) {
        const int X = x0 >> 1, Y = y0 >> 1;
        put(1, X, Y, ma);
        put(1, X + 1, Y, mb);
    }
    // levels 2 and 3 inside the wave (a wave holds 4 rows of 16 threads: the level-1 texels of
    // 64 x 8 pixels): each level's 2x2 maximum from the lanes 1 / 16 / 32 apart (ds_bpermute, no
    // barrier); only level 3 crosses waves, through LDS, and wave 0 reduces levels 4-6 the same way
    // -- one workgroup barrier instead of five (the prep of a shard's batch is replicated on every
    // rank: its workgroups are a fixed share of the launch's tail)
    float m2 = fmaxf(ma, mb);
    m2 = fmaxf(m2, __shfl_down(m2, 16));  // rows r, r + 1 (r even)
    if (act && (r & 1) == 0) put(2, tx * 16 + c, ty * 16 + (r >> 1), m2);
    float m3 = fmaxf(m2, __shfl_down(m2, 1));
    m3 = fmaxf(m3, __shfl_down(m3, 32));  // level-2 rows r/2, r/2 + 1 (r % 4 == 0), columns c, c + 1
    if (act && (r & 3) == 0 && (c & 1) == 0) {
        put(3, tx * 8 + (c >> 1), ty * 8 + (r >> 2), m3);
        sa[r >> 2][c >> 1] = m3;
    }
    __syncthreads();
    if (t < 64) {  // wave 0: the tile's 8 x 8 level-3 texels, lane = y * 8 + x
        const int lx = t & 7, ly = t >> 3;
        float m = sa[ly][lx];
        m = fmaxf(m, __shfl_down(m, 1));
        m = fmaxf(m, __shfl_down(m, 8));
        if ((lx & 1) == 0 && (ly & 1) == 0) put(4, tx * 4 + (lx >> 1), ty * 4 + (ly >> 1), m);
        m = fmaxf(m, __shfl_down(m, 2));
        m = fmaxf(m, __shfl_down(m, 16));
        if ((lx & 3) == 0 && (ly & 3) == 0) put(5, tx * 2 + (lx >> 2), ty * 2 + (ly >> 2), m);
        m = fmaxf(m, __shfl_down(m, 4));
        m = fmaxf(m, __shfl_down(m, 32));
        if (t == 0) put(6, tx, ty, m);
    }
    (void)sb;
}

template <int DK = 0>
__global__ __launch_bounds__(512) void k_prep_vec(Batch bt, unsigned int* count) {
    __shared__ float sa[32][33];
    __shared__ float sb[32][33];
    prep_vec_tile<DK>(bt, count, blockIdx.x, blockIdx.y, blockIdx.z, sa, sb);
}

template <int DK, int CK>
__global__ __launch_bounds__(1024) void k_prep(Batch bt, unsigned int* count) {
    __shared__ float sa[32][33];
    __shared__ float sb[32][33];
    const Frame& fr = bt.f[blockIdx.z];
    float* pyr = (float*)fr.pyr;
    unsigned* rgbx = (unsigned*)fr.rgbx;
    const int t = threadIdx.x, r = t >> 5, c = t & 31;
    if (count && t < kCountWords && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) coh_store(count + t, 0u);
    const int x0 = blockIdx.x * 64 + c * 2, y0 = blockIdx.y * 64 + r * 2;
    float m1 = 0.0f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const int x = x0 + dx, y = y0 + dy;
            if (x < fr.W && y < fr.H) {
                const int p = y * fr.W + x;
                float d;
                if (DK == 0) {
                    unsigned v = ((const unsigned short*)fr.depth_src)[p];
                    if (fr.depth_mask) {  // the demos' depth_im[depth_im == 65.535] = 0
                        v = (v == 65535u) ? 0u : v;
                        fr.depth_mask[p] = (unsigned short)v;
                    }
                    d = (float)v * 1e-3f;
                } else {
                    d = (float)((const double*)fr.depth_src)[p];
                }
                if (CK == 0 && rgbx) {
                    const unsigned char* q = (const unsigned char*)fr.color + 3 * (size_t)p;
                    const unsigned c = (unsigned)q[0] | ((unsigned)q[1] << 8) | ((unsigned)q[2] << 16);
                    rgbx[p] = c;
                }
                m1 = fmaxf(m1, (float)d);
            }
        }
    {
        const int X = (x0 >> 1), Y = (y0 >> 1);
        if (X < bt.pg.w[1] && Y < bt.pg.h[1]) pyr[bt.pg.off[1] + Y * bt.pg.w[1] + X] = m1;
    }
    sa[r][c] = m1;
    __syncthreads();
    pyr_level<0>(bt.pg, pyr, 2, sa, sb, 16);
    __syncthreads();
    pyr_level<0>(bt.pg, pyr, 3, sb, sa, 8);
    __syncthreads();
    pyr_level<0>(bt.pg, pyr, 4, sa, sb, 4);
    __syncthreads();
    pyr_level<0>(bt.pg, pyr, 5, sb, sa, 2);
    __syncthreads();
    pyr_level<0>(bt.pg, pyr, 6, sa, sb, 1);
}

// ---------------------------------------------------------------------------------------------
// One launch of the dense grid's three-stage software pipeline.  Launch k runs
//   workgroups [0, gi)          integrate batch k   (list set k, written by launch k-1),
//   workgroups [gi, gi + gc)    cull batch k+1      (one superbrick each; pyramid of launch k-1),
//   the rest                    prep batch k+2      (one 64x64 tile of one frame each).
// The stages touch disjoint buffer sets (batch j uses set j % 3) and every input of a stage was
// written by an earlier launch on the same stream, so no workgroup ever waits for another.  The
// integrate workgroups come first in dispatch order; the cull and prep workgroups take the CUs
// its tail frees.  One launch per batch replaces three kernels and the gaps between them.
// ---------------------------------------------------------------------------------------------
// Fused workgroups: the integrate's waves share one dynamic item pool per workgroup, so larger
// workgroups balance better; the cull and prep stages use the first 512 threads.
#ifndef TSDF_FUSED_WG
#define TSDF_FUSED_WG 768  // dense: 12 waves, 2 per CU at 6 waves/SIMD (+0.8 % over 512)
#endif
#ifndef TSDF_FUSED_HASH_WG  // hash: 768 too (12 waves, 2 per CU): -3.6 % per launch against 512 on
#define TSDF_FUSED_HASH_WG 768  // the 250-step window, even on the driver window (profiles/r04_h2/)
#endif
constexpr int kFusedWG = TSDF_FUSED_WG, kFusedHashWG = TSDF_FUSED_HASH_WG;
static_assert(kFusedWG >= kCullWG && kFusedHashWG >= kCullWG && kFusedWG % 64 == 0 && kFusedHashWG % 64 == 0,
              "a cull workgroup is one wave per frame of the batch");
struct Stage {
    const ListEntry* list_i;  // integrate: list and count of batch k
    unsigned int* count_i;
    ListEntry* list_c;        // cull: list and count of batch k+1
    unsigned int* count_c;
    unsigned int* count_p;   // prep: count of batch k+2 (reset for its cull)
    int gi, gc;              // integrate / cull workgroups
    int cg;                  // superbricks per cull workgroup (<= kCullGMax)
    int ptx, pty;            // prep tiles per frame (x, y)
    long long seq;           // hash: launch number for the pool report (Table::rb)
    int* res_i;              // hash: per-brick claim words of batch k (integrate) and k+1 (cull)
    int* res_c;
    unsigned* done;          // hash: arrival counter of the launch's integrate and cull workgroups
};

#ifdef TSDF_WG_TIMES
// Diagnostic builds only (tools/gpu/wg_times.py): per workgroup of the last full fused launch, its
// start and end (s_memrealtime, 100 MHz) and role << 32 | the list items its waves took (role 0
// integrate, 1 cull, 2 prep).
constexpr int kWgTimes = 16384;
__device__ unsigned long long g_wg_times[4][kWgTimes];  // start, end, role << 32 | items, XCC << 32 | HW_ID
__device__ inline unsigned long long wg_place() {  // where the workgroup runs: XCC id << 32 | HW_ID (CU, SE, ...)
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return ((unsigned long long)xcc << 32) | hw;
}
#endif
// The dense fused launch's arguments as one struct (the kernel addresses its kernarg copy).
struct FusedArgs {
    Vol v;
    Batch bi, bc, bp;
    Pool pool;
    unsigned long long* stats;
    Stage sg;
};
typedef const __attribute__((address_space(4))) FusedArgs* FusedArgsP;

template <bool OW1, int NZ, int DK = 0, bool CU = false>
__global__ __launch_bounds__(kFusedWG) __attribute__((amdgpu_waves_per_eu(TSDF_DENSE_WAVES))) void k_fused(FusedArgs a) {
    const FusedArgsP A = (FusedArgsP)__builtin_amdgcn_kernarg_segment_ptr();
    const Vol& v = *(const Vol*)opaque(&A->v);
    const Pool& pool = *(const Pool*)opaque(&A->pool);
    const Batch &bi = a.bi, &bc = a.bc, &bp = a.bp;
    unsigned long long* const stats = a.stats;
    const Stage& sg = a.sg;
    // integrate: RN(1/n) table; cull: per-brick frame masks; prep: two pyramid tiles
    __shared__ double s_buf[kRcpTab];
    __shared__ unsigned long long s_stat[kNStat];
    __shared__ unsigned s_next;
    const int tid = threadIdx.x, b = blockIdx.x;
    const Table no_table{};
#ifdef TSDF_WG_TIMES
    // (launches with all three stages only: the steady state of a call)
    const bool rec = sg.gi > 0 && sg.gc > 0 && (int)gridDim.x > sg.gi + sg.gc && b < kWgTimes;
    if (tid == 0 && rec) g_wg_times[0][b] = __builtin_amdgcn_s_memrealtime();
#endif
    if (b < sg.gi) {
        if (tid < kNStat) s_stat[tid] = 0;
        if (tid == 0) s_next = 0;
        if (OW1)
            for (int i = tid; i < kRcpTab / 2; i += kFusedWG) ((double2*)s_buf)[i] = ((const double2*)v.rcp)[i];
        __syncthreads();
        constexpr int wpg = kFusedWG / 64;
        integrate_list<false, DK, 0, OW1, NZ, CU>(v, bi, pool, no_table, sg.list_i, sg.count_i, 0,
                                             b * wpg + (tid >> 6), sg.gi * wpg, s_stat,
                                             OW1 ? s_buf : nullptr, &s_next, b, sg.gi);
        __syncthreads();
        flush_stats(s_stat, stats);
    } else if (b < sg.gi + sg.gc) {
        cull_superbrick<false>(v, bc, no_table, sg.list_c, sg.count_c, stats, b - sg.gi, (unsigned*)s_buf,
                               s_stat, nullptr, sg.cg);
    } else {
        const int t = b - sg.gi - sg.gc, per = sg.ptx * sg.pty;
        const int f = t / per, r = t - f * per;
        float(*sa)[33] = (float(*)[33])s_buf;
        prep_vec_tile<DK>(bp, sg.count_p, r % sg.ptx, r / sg.ptx, f, sa, sa + 32);
    }
#ifdef TSDF_WG_TIMES
    __syncthreads();
    if (tid == 0 && rec) {
        g_wg_times[1][b] = __builtin_amdgcn_s_memrealtime();
        g_wg_times[3][b] = wg_place();
        g_wg_times[2][b] = ((unsigned long long)(b < sg.gi ? 0 : b < sg.gi + sg.gc ? 1 : 2) << 32) |
                           (b < sg.gi ? s_next : 0u);
    }
#endif
}

// Fold one launch's allocations (PoolState::cursor) into the free list / bump pointer (the
// hash's k_commit, also run by the last integrate workgroup of a fused hash launch).
__device__ inline void commit_pool(PoolState* st, long long max_blocks, PoolReport* rb = nullptr,
                                   long long seq = -1, const unsigned* count = nullptr) {
    const long long used = coh_load(&st->cursor);
    const long long nf = coh_load(&st->free_count);
    const long long cons = used < nf ? used : nf;
    long long top = coh_load(&st->pool_top) + (used - cons);
    top = top < max_blocks ? top : max_blocks;
    coh_store(&st->free_count, nf - cons);
    coh_store(&st->pool_top, top);
    coh_store(&st->cursor, 0ll);
    if (rb && seq >= 0) {  // report to the host (vector stores to fine-grained host memory)
        PoolReport* r = rb + (seq % kReports);
        __hip_atomic_store(&r->pool_top, top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&r->free_count, nf - cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&r->n_overflow, coh_load(&st->n_overflow), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&r->tombs, coh_load(&st->tombs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        long long listed = 0;  // the cost-class sub-list lengths of the list given (the allocating one)
        if (count)
            for (int c = 1; c <= kMaxBatch; ++c) listed += coh_load(&((unsigned*)count)[c]);
        __hip_atomic_store(&r->listed, listed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&r->seq, seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The voxel hash's three-stage launch (u16 + RGB8, obs_weight 1 as HashTable.integrate): as
// k_fused, with the hash integrate (z-half waves on the blocks the previous launch's cull found or
// inserted) and a cull that finds or inserts the blocks of the next batch; the pool commit of the
// cull's allocations is done by the integrate or cull workgroup that finishes last (an arrival
// counter; every workgroup's allocations are complete before it arrives).
#ifndef TSDF_FUSED_HASH_WAVES
#define TSDF_FUSED_HASH_WAVES 6
#endif
// The launch's arguments as one struct, so that the kernel can address its own copy in the
// kernarg segment (fused_args).
struct FusedHashArgs {
    Vol v;
    Batch bi, bc, bp;
    Pool pool;
    Table tab;
    unsigned long long* stats;
    Stage sg;
};

template <int DK = 0, bool CU = false>
__global__ __launch_bounds__(kFusedHashWG) __attribute__((amdgpu_waves_per_eu(TSDF_FUSED_HASH_WAVES))) void k_fused_hash(
        FusedHashArgs a) {
    typedef const __attribute__((address_space(4))) FusedHashArgs* ArgsP;
    const ArgsP A = (ArgsP)__builtin_amdgcn_kernarg_segment_ptr();
    const Table& tab = *(const Table*)opaque(&A->tab);
    const Vol& v = *(const Vol*)opaque(&A->v);
    const Pool& pool = *(const Pool*)opaque(&A->pool);
    const Batch &bi = a.bi, &bc = a.bc, &bp = a.bp;
    unsigned long long* const stats = a.stats;
    const Stage& sg = a.sg;
    __shared__ double s_buf[kRcpTab];
    __shared__ unsigned long long s_stat[kNStat];
    __shared__ int s_last;
    __shared__ unsigned s_next;
    const int tid = threadIdx.x, b = blockIdx.x;
#ifdef TSDF_WG_TIMES
    const bool rec = sg.gi > 0 && sg.gc > 0 && (int)gridDim.x > sg.gi + sg.gc && b < kWgTimes;
    if (tid == 0 && rec) g_wg_times[0][b] = __builtin_amdgcn_s_memrealtime();
#endif
    if (b < sg.gi) {
        if (tid < kNStat) s_stat[tid] = 0;
        if (tid == 0) s_next = 0;
        for (int i = tid; i < kRcpTab / 2; i += kFusedHashWG) ((double2*)s_buf)[i] = ((const double2*)v.rcp)[i];
        __syncthreads();
        constexpr int wpg = kFusedHashWG / 64;
        integrate_list<true, DK, 0, true, 4, CU>(v, bi, pool, tab, sg.list_i, sg.count_i, 0, b * wpg + (tid >> 6),
                                            sg.gi * wpg, s_stat, s_buf, &s_next, b, sg.gi, sg.res_i);
        __syncthreads();
        flush_stats(s_stat, stats);
    } else if (b < sg.gi + sg.gc) {
        if (tab.owned)
            cull_owned<true>(v, bc, tab, sg.list_c, sg.count_c, stats, b - sg.gi, (unsigned*)s_buf, s_stat, sg.res_c,
                             &pool);
        else
            cull_superbrick<true, true>(v, bc, tab, sg.list_c, sg.count_c, stats, b - sg.gi, (unsigned*)s_buf,
                                        s_stat, sg.res_c, sg.cg, &pool);
    }
    if (b < sg.gi + sg.gc) {  // the last integrate / cull workgroup commits the launch's allocations
        if (tid == 0) {
            __threadfence();  // this workgroup's allocations and stores before its arrival
            s_last = atomicAdd(sg.done, 1u) == (unsigned)(sg.gi + sg.gc) - 1;
        }
        __syncthreads();
        if (s_last && tid == 0) {
            __threadfence();
            commit_pool(tab.st, tab.max_blocks, tab.rb, sg.seq, sg.gc ? sg.count_c : nullptr);
        }
    } else {
        const int t = b - sg.gi - sg.gc, per = sg.ptx * sg.pty;
        const int f = t / per, r = t - f * per;
        float(*sa)[33] = (float(*)[33])s_buf;
        prep_vec_tile<DK>(bp, sg.count_p, r % sg.ptx, r / sg.ptx, f, sa, sa + 32);
    }
#ifdef TSDF_WG_TIMES
    __syncthreads();
    if (tid == 0 && rec) {
        g_wg_times[1][b] = __builtin_amdgcn_s_memrealtime();
        g_wg_times[3][b] = wg_place();
        g_wg_times[2][b] = ((unsigned long long)(b < sg.gi ? 0 : b < sg.gi + sg.gc ? 1 : 2) << 32) |
                           (b < sg.gi ? s_next : 0u);
    }
#endif
}

}  // namespace tsdf
