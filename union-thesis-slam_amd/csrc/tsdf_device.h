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

namespace tsdf {

constexpr int kBrickEdge = 8;
constexpr int kBrickVox = 512;      // 8^3 voxels; brick-local index = z*64 + x*8 + y
constexpr int kWG = 256;            // threads per workgroup (4 waves of 64)
constexpr int kPyrLevels = 6;       // max-depth pyramid levels 1..6 (2x2 .. 64x64 pixels)
constexpr int kStatSpread = 64;     // counters are spread over 64 words (no hot atomic word)
constexpr unsigned long long kEmpty = ~0ull;
constexpr unsigned long long kTomb = ~0ull - 1ull;

enum Stat { ST_VOXELS = 0, ST_VISITED, ST_TOUCHED, ST_ALLOC, ST_PROBE, ST_LOOKUPS, ST_OVERFLOW,
            ST_PROBE_MAX, kNStat };

// Volume geometry (by value in kernel arguments -> scalar registers).
struct Vol {
    int dims[3];    // voxels of this shard
    int off[3];     // global voxel index of local (0,0,0)
    int nb[3];      // bricks per axis (ceil(dims/8))
    int shard, n_shards;
    float origin[3];
    double vs, trunc;
};

// Per-frame constants (by value).
struct Frame {
    double T[12];             // rows 0..2 of inv(cam_pose), row-major
    double fx, fy, cx, cy;    // f64(f32(K))  (cam2pix casts intr to float32, grid_fusion.py:190)
    double ow;                // obs_weight as a Python float (f64)
    float ow32;               // the same weight as NumPy's weak-scalar f32 (colour blend)
    int H, W;
    const void* depth;
    const void* color;
    const float* pyr;         // max-depth pyramid (metres), levels 1..6 concatenated
    int pyr_off[kPyrLevels + 1];
    int pyr_w[kPyrLevels + 1];
    int pyr_h[kPyrLevels + 1];
};

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
};

struct Table {
    unsigned long long* keys;   // capacity slots; kEmpty / kTomb / packed brick key
    int* vals;                  // pool block of each slot
    unsigned long long* occ;    // [max_blocks][8] voxel-entry bits (word = z, bit = x*8+y)
    int* free_list;
    int* overflow;              // brick ids skipped this launch
    PoolState* st;
    long long capacity;
    long long max_blocks;
    int overflow_cap;
    int int_bits;               // 64: NumPy int64; 32: wrapping int32 (author's Windows run)
};

// hash_function (hash_fusion.py:182-190): ((x*P1) ^ (y*P2) ^ (z*P3)) floor-mod n.
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
    long long m = h % n;
    return m < 0 ? m + n : m;
}

__host__ __device__ inline unsigned long long pack_key(int bx, int by, int bz) {
    return (unsigned long long)bx | ((unsigned long long)by << 21) | ((unsigned long long)bz << 42);
}

__device__ inline int lane_id() { return threadIdx.x & 63; }

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

// Depth in metres at pixel p, exactly as NumPy computes it: astype(float) / 1000.
template <int DK>
__device__ inline double depth_at(const Frame& fr, int p) {
    if (DK == 0) {
        const unsigned short mm = ((const unsigned short*)fr.depth)[p];
        return (double)mm / 1000.0;
    } else {
        return ((const double*)fr.depth)[p];
    }
}

// World position of a global voxel index (vox2world, grid_fusion.py:170-181):
// f32( f64(origin_f32) + vs * f64(f32(idx)) ); idx < 2^24 so f32(idx) is exact.
__device__ inline double vox_world(float origin, double vs, int g) {
    return (double)(float)((double)origin + vs * (double)g);
}

// Conservative cull of one brick against the frame.  True = some voxel of the brick MAY pass
// the reference's masks (grid_fusion.py:273-290).  Never drops a brick that has a valid voxel:
// the box of voxel centres is projected exactly (f64), its pixel bbox grown by one pixel, and
// the depth test is taken against the max depth over that bbox with a 1 mm slack.
__device__ inline bool cull_brick(const Vol& v, const Frame& fr, int bx, int by, int bz) {
    int lo[3] = {bx * kBrickEdge, by * kBrickEdge, bz * kBrickEdge};
    int hi[3];
    for (int a = 0; a < 3; ++a) {
        hi[a] = min(lo[a] + kBrickEdge - 1, v.dims[a] - 1) + v.off[a];
        lo[a] += v.off[a];
    }
    double zmin = 1e300, zmax = -1e300, umin = 1e300, umax = -1e300, vmin = 1e300, vmax = -1e300;
    for (int c = 0; c < 8; ++c) {
        const double px = (double)v.origin[0] + v.vs * (double)((c & 1) ? hi[0] : lo[0]);
        const double py = (double)v.origin[1] + v.vs * (double)((c & 2) ? hi[1] : lo[1]);
        const double pz = (double)v.origin[2] + v.vs * (double)((c & 4) ? hi[2] : lo[2]);
        const double x = fr.T[0] * px + fr.T[1] * py + fr.T[2] * pz + fr.T[3];
        const double y = fr.T[4] * px + fr.T[5] * py + fr.T[6] * pz + fr.T[7];
        const double z = fr.T[8] * px + fr.T[9] * py + fr.T[10] * pz + fr.T[11];
        zmin = fmin(zmin, z);
        zmax = fmax(zmax, z);
        const double iz = 1.0 / fmax(z, 1e-9);
        const double u = fr.fx * x * iz + fr.cx, w = fr.fy * y * iz + fr.cy;
        umin = fmin(umin, u); umax = fmax(umax, u);
        vmin = fmin(vmin, w); vmax = fmax(vmax, w);
    }
    if (zmax < -1e-4) return false;  // every voxel has z <= 0
    int u0 = 0, u1 = fr.W - 1, v0 = 0, v1 = fr.H - 1;
    if (zmin > 0.02) {  // whole brick in front of the camera: projected hull is convex
        const double fu0 = floor(umin) - 1.0, fu1 = ceil(umax) + 1.0;
        const double fv0 = floor(vmin) - 1.0, fv1 = ceil(vmax) + 1.0;
        if (fu1 < 0.0 || fv1 < 0.0 || fu0 > (double)(fr.W - 1) || fv0 > (double)(fr.H - 1))
            return false;
        u0 = (int)fmax(fu0, 0.0); u1 = (int)fmin(fu1, (double)(fr.W - 1));
        v0 = (int)fmax(fv0, 0.0); v1 = (int)fmin(fv1, (double)(fr.H - 1));
    }
    // max depth over the bbox from the smallest pyramid level where it spans <= 4x4 texels
    int L = 1;
    while (L < kPyrLevels && (((u1 >> L) - (u0 >> L)) > 3 || ((v1 >> L) - (v0 >> L)) > 3)) ++L;
    const float need = (float)(zmin - v.trunc) - 1e-3f;
    const float* lvl = fr.pyr + fr.pyr_off[L];
    const int wl = fr.pyr_w[L];
    float dmax = 0.0f;
    for (int ty = v0 >> L; ty <= (v1 >> L); ++ty)
        for (int tx = u0 >> L; tx <= (u1 >> L); ++tx) {
            dmax = fmaxf(dmax, lvl[ty * wl + tx]);
        }
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
        const unsigned long long kk = coh_load(&t.keys[s]);
        const unsigned long long hit = __ballot(kk == key);
        if (hit) {
            const int l = __ffsll((long long)hit) - 1;
            slot_out = __shfl(s, l);
            probe = scanned + l;
            return coh_load(&t.vals[slot_out]);
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


// ---------------------------------------------------------------------------------------------
// Per-brick integrate: one wave, lane (x,y) = (lane>>3, lane&7) walks z = 0..7, so the
// x/y part of the camera transform is computed once per column and every z-step's 64 loads
// and stores are one contiguous 256-B segment of the brick (brick-local index z*64 + lane).
// ---------------------------------------------------------------------------------------------
template <bool HASH, int DK, int CK>
__device__ inline void integrate_brick(const Vol& v, const Frame& fr, const Pool& pool,
                                       const Table& tab, int b, unsigned long long* s_stat) {
    const int lane = lane_id();
    const int nb12 = v.nb[1] * v.nb[2];
    const int bx = b / nb12;
    const int rem = b - bx * nb12;
    const int by = rem / v.nb[2];
    const int bz = rem - by * v.nb[2];
    const int lx = bx * kBrickEdge + (lane >> 3);
    const int ly = by * kBrickEdge + (lane & 7);
    const bool col_in = lx < v.dims[0] && ly < v.dims[1];
    // vox2world + the x/y terms of OpenBLAS's dgemm chain (grid_fusion.py:170-181, 363-368)
    const double px = vox_world(v.origin[0], v.vs, v.off[0] + lx);
    const double py = vox_world(v.origin[1], v.vs, v.off[1] + ly);
    const double a0 = fma(fr.T[1], py, fr.T[0] * px);
    const double a1 = fma(fr.T[5], py, fr.T[4] * px);
    const double a2 = fma(fr.T[9], py, fr.T[8] * px);

    unsigned vmask = 0;
    int pix[kBrickEdge];
    double dist[kBrickEdge];
#pragma unroll
    for (int k = 0; k < kBrickEdge; ++k) {
        pix[k] = 0;
        dist[k] = 0.0;
        const int lz = bz * kBrickEdge + k;
        if (!col_in || lz >= v.dims[2]) continue;
        const double pz = vox_world(v.origin[2], v.vs, v.off[2] + lz);
        const double z = fr.T[11] + fma(fr.T[10], pz, a2);  // fma(T3, 1, s) == T3 + s
        if (!(z > 0.0)) continue;
        const double x = fr.T[3] + fma(fr.T[2], pz, a0);
        const double y = fr.T[7] + fma(fr.T[6], pz, a1);
        // cam2pix (grid_fusion.py:195-196): mul, div, add, round-half-even
        const double u = rint((x * fr.fx) / z + fr.cx);
        const double w = rint((y * fr.fy) / z + fr.cy);
        if (!(u >= 0.0 && u < (double)fr.W && w >= 0.0 && w < (double)fr.H)) continue;
        const int p = (int)w * fr.W + (int)u;
        // depth test (grid_fusion.py:278-286)
        const double d = depth_at<DK>(fr, p);
        const double diff = d - z;
        if (!(d > 0.0 && diff >= -v.trunc)) continue;
        const double dd = diff / v.trunc;
        dist[k] = dd > 1.0 ? 1.0 : dd;  // np.minimum(1, .)
        pix[k] = p;
        vmask |= 1u << k;
    }
    if (__ballot(vmask != 0) == 0) return;

    long long blk = b;
    bool is_new = false;
    if (HASH) {
        long long slot = 0, probe = 0;
        const unsigned long long key = pack_key(bx, by, bz);
        const long long home = ref_hash(bx, by, bz, tab.capacity, tab.int_bits);
        const int r = table_find_or_insert(tab, key, home, true, is_new, slot, probe);
        if (r < 0) {  // no space: skip the whole brick; the host grows the table and re-runs it
            if (lane == 0) {
                const unsigned long long o = atomicAdd((unsigned long long*)&tab.st->n_overflow, 1ull);
                if ((long long)o < tab.overflow_cap) tab.overflow[o] = b;
                atomicAdd(&s_stat[ST_OVERFLOW], 1ull);
            }
            return;
        }
        blk = r;
        if (lane == 0) {
            atomicAdd(&s_stat[ST_LOOKUPS], 1ull);
            atomicAdd(&s_stat[ST_PROBE], (unsigned long long)probe);
            atomicMax(&s_stat[ST_PROBE_MAX], (unsigned long long)probe);
            if (is_new) atomicAdd(&s_stat[ST_ALLOC], 1ull);
        }
    }

    const size_t base = (size_t)blk * kBrickVox + lane;
    int nupd = 0;
#pragma unroll
    for (int k = 0; k < kBrickEdge; ++k) {
        const size_t idx = base + (size_t)k * 64;
        if ((vmask >> k) & 1u) {
            float w_old = 0.0f, t_old = 1.0f, c_old = 0.0f;
            if (!(HASH && is_new)) {
                w_old = pool.weight[idx];
                t_old = pool.tsdf[idx];
                c_old = pool.color[idx];
            }
            // integrate_tsdf (grid_fusion.py:207-212): w f32 <- f64 add; f32 product; f64 average
            const float w_new = (float)((double)w_old + fr.ow);
            const float wt = w_old * t_old;
            const float t_new = (float)(((double)wt + fr.ow * dist[k]) / (double)w_new);
            // colour (grid_fusion.py:302-314): float32 throughout, round half to even
            const float ob = floorf(c_old / 65536.0f);
            const float og = floorf((c_old - ob * 65536.0f) / 256.0f);
            const float orr = c_old - ob * 65536.0f - og * 256.0f;
            float nb, ng, nr;
            if (CK == 0) {  // uint8 RGB: the fold/decode round trip is exact
                const unsigned char* c = (const unsigned char*)fr.color + 3 * (size_t)pix[k];
                nr = (float)c[0];
                ng = (float)c[1];
                nb = (float)c[2];
            } else {
                const float nc = ((const float*)fr.color)[pix[k]];
                nb = floorf(nc / 65536.0f);
                ng = floorf((nc - nb * 65536.0f) / 256.0f);
                nr = nc - nb * 65536.0f - ng * 256.0f;
            }
            const float cb = fminf(255.0f, rintf((w_old * ob + fr.ow32 * nb) / w_new));
            const float cg = fminf(255.0f, rintf((w_old * og + fr.ow32 * ng) / w_new));
            const float cr = fminf(255.0f, rintf((w_old * orr + fr.ow32 * nr) / w_new));
            pool.weight[idx] = w_new;
            pool.tsdf[idx] = t_new;
            pool.color[idx] = cb * 65536.0f + cg * 256.0f + cr;
            ++nupd;
        } else if (HASH && is_new) {  // first touch of a pool block: initialise it
            pool.weight[idx] = 0.0f;
            pool.tsdf[idx] = 1.0f;
            pool.color[idx] = 0.0f;
        }
    }
    if (HASH) {  // voxel-entry bits: word z, bit (x*8+y); this wave owns the block this launch
        unsigned long long mine = 0;
#pragma unroll
        for (int k = 0; k < kBrickEdge; ++k) {
            const unsigned long long m = __ballot((vmask >> k) & 1u);
            if (lane == k) mine = m;
        }
        if (lane < kBrickEdge) {
            unsigned long long* o = tab.occ + (size_t)blk * kBrickEdge + lane;
            if (is_new) coh_store(o, mine);
            else if (mine) atomicOr(o, mine);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nupd += __shfl_xor(nupd, off);
    if (lane == 0) {
        atomicAdd(&s_stat[ST_VOXELS], (unsigned long long)nupd);
        atomicAdd(&s_stat[ST_TOUCHED], 1ull);
    }
}

// Fused cull + integrate.  Workgroup g owns bricks {g + t*G : t < 256} (G = gridDim.x): an
// interleaved sample of the whole volume, so every workgroup gets a similar share of the
// visible bricks without a global work queue.  With `list` the bricks come from it instead
// (hash overflow re-run).
template <bool HASH, int DK, int CK>
__global__ __launch_bounds__(kWG) void k_integrate(Vol v, Frame fr, Pool pool, Table tab,
                                                  unsigned long long* stats, const int* list,
                                                  int n_list) {
    __shared__ int s_list[kWG];
    __shared__ int s_cnt[kWG / 64];
    __shared__ unsigned long long s_stat[kNStat];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kNStat) s_stat[tid] = 0;
    bool keep = false;
    int b = 0;
    if (list) {
        const long long e = (long long)blockIdx.x * kWG + tid;
        if (e < n_list) {
            b = list[e];
            keep = true;
        }
    } else {
        const long long nbricks = (long long)v.nb[0] * v.nb[1] * v.nb[2];
        const long long e = (long long)blockIdx.x + (long long)tid * gridDim.x;
        if (e < nbricks) {
            b = (int)e;
            const int nb12 = v.nb[1] * v.nb[2];
            const int bx = b / nb12, rem = b - bx * nb12, by = rem / v.nb[2], bz = rem - by * v.nb[2];
            keep = true;
            if (HASH && v.n_shards > 1) {  // bucket-range ownership
                const long long home = ref_hash(bx, by, bz, tab.capacity, tab.int_bits);
                keep = (int)((home * v.n_shards) / tab.capacity) == v.shard;
            }
            if (keep) keep = cull_brick(v, fr, bx, by, bz);
        }
    }
    // compact the survivors: wave ballot + LDS prefix over the 4 waves
    const unsigned long long m = __ballot(keep);
    if (lane == 0) s_cnt[wave] = __popcll(m);
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWG / 64; ++w) {
        const int c = s_cnt[w];
        base += (w < wave) ? c : 0;
        total += c;
    }
    if (keep) s_list[base + __popcll(m & ((1ull << lane) - 1ull))] = b;
    __syncthreads();
    for (int e = wave; e < total; e += kWG / 64)
        integrate_brick<HASH, DK, CK>(v, fr, pool, tab, s_list[e], s_stat);
    if (tid == 0) atomicAdd(&s_stat[ST_VISITED], (unsigned long long)total);
    __syncthreads();
    if (tid < kNStat && s_stat[tid]) {
        unsigned long long* dst = stats + tid * kStatSpread + (blockIdx.x & (kStatSpread - 1));
        if (tid == ST_PROBE_MAX) atomicMax(dst, s_stat[tid]);
        else atomicAdd(dst, s_stat[tid]);
    }
}

// Max-depth pyramid, levels 1..6 (texel = max over a 2^L x 2^L pixel block, metres, 0 for
// invalid/outside).  One workgroup per 64x64 tile; each thread reduces a 4x4 patch.
template <int DK>
__global__ __launch_bounds__(kWG) void k_pyramid(Frame fr, float* pyr) {
    __shared__ float s2[16][16];
    __shared__ float s3[8][8];
    __shared__ float s4[4][4];
    __shared__ float s5[2][2];
    const int t = threadIdx.x, r = t >> 4, c = t & 15;
    const int x0 = blockIdx.x * 64 + c * 4, y0 = blockIdx.y * 64 + r * 4;
    float m2 = 0.0f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            float m1 = 0.0f;
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    const int x = x0 + q * 2 + dx, y = y0 + a * 2 + dy;
                    if (x < fr.W && y < fr.H) {
                        const int p = y * fr.W + x;
                        const float d = (DK == 0) ? (float)((const unsigned short*)fr.depth)[p] * 1e-3f
                                                  : (float)((const double*)fr.depth)[p];
                        m1 = fmaxf(m1, d);
                    }
                }
            const int tx1 = (x0 >> 1) + q, ty1 = (y0 >> 1) + a;
            if (tx1 < fr.pyr_w[1] && ty1 < fr.pyr_h[1]) pyr[fr.pyr_off[1] + ty1 * fr.pyr_w[1] + tx1] = m1;
            m2 = fmaxf(m2, m1);
        }
    if ((x0 >> 2) < fr.pyr_w[2] && (y0 >> 2) < fr.pyr_h[2])
        pyr[fr.pyr_off[2] + (y0 >> 2) * fr.pyr_w[2] + (x0 >> 2)] = m2;
    s2[r][c] = m2;
    __syncthreads();
    if (t < 64) {
        const int rr = t >> 3, cc = t & 7;
        const float m = fmaxf(fmaxf(s2[2 * rr][2 * cc], s2[2 * rr][2 * cc + 1]),
                              fmaxf(s2[2 * rr + 1][2 * cc], s2[2 * rr + 1][2 * cc + 1]));
        s3[rr][cc] = m;
        const int X = blockIdx.x * 8 + cc, Y = blockIdx.y * 8 + rr;
        if (X < fr.pyr_w[3] && Y < fr.pyr_h[3]) pyr[fr.pyr_off[3] + Y * fr.pyr_w[3] + X] = m;
    }
    __syncthreads();
    if (t < 16) {
        const int rr = t >> 2, cc = t & 3;
        const float m = fmaxf(fmaxf(s3[2 * rr][2 * cc], s3[2 * rr][2 * cc + 1]),
                              fmaxf(s3[2 * rr + 1][2 * cc], s3[2 * rr + 1][2 * cc + 1]));
        s4[rr][cc] = m;
        const int X = blockIdx.x * 4 + cc, Y = blockIdx.y * 4 + rr;
        if (X < fr.pyr_w[4] && Y < fr.pyr_h[4]) pyr[fr.pyr_off[4] + Y * fr.pyr_w[4] + X] = m;
    }
    __syncthreads();
    if (t < 4) {
        const int rr = t >> 1, cc = t & 1;
        const float m = fmaxf(fmaxf(s4[2 * rr][2 * cc], s4[2 * rr][2 * cc + 1]),
                              fmaxf(s4[2 * rr + 1][2 * cc], s4[2 * rr + 1][2 * cc + 1]));
        s5[rr][cc] = m;
        const int X = blockIdx.x * 2 + cc, Y = blockIdx.y * 2 + rr;
        if (X < fr.pyr_w[5] && Y < fr.pyr_h[5]) pyr[fr.pyr_off[5] + Y * fr.pyr_w[5] + X] = m;
    }
    __syncthreads();
    if (t == 0) {
        const float m = fmaxf(fmaxf(s5[0][0], s5[0][1]), fmaxf(s5[1][0], s5[1][1]));
        const int X = blockIdx.x, Y = blockIdx.y;
        if (X < fr.pyr_w[6] && Y < fr.pyr_h[6]) pyr[fr.pyr_off[6] + Y * fr.pyr_w[6] + X] = m;
    }
}

}  // namespace tsdf
