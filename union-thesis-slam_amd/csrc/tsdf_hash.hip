// tsdf_hash.hip -- voxel-hash map store: the MI355X replacement of HashTable
// (hash_fusion.py:29-507).
//
// Keys are 8^3 voxel blocks (bx,by,bz) packed into 63 bits; the home slot is the reference's
// hash_function of the block coordinates (hash_fusion.py:182-190).  Open addressing with
// linear probing over `capacity` slots; keys go EMPTY -> key by CAS only, removal leaves a
// tombstone; a resize rehashes every live key (double_table_size, hash_fusion.py:414-437).
// Blocks come from a pool (SoA f32 bricks like the dense grid) with a bump allocator and a
// free list.  A voxel "entry" (count_num_hash_entries, get_hash_entry) is one bit of the
// block's 512-bit occupancy mask, set by integrate or by an explicit insert.
#include <algorithm>
#include <vector>
#include <climits>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "tsdf_host.h"

#ifdef TSDF_HOST_TIMES
// (diagnostic builds, tools/gpu/dropin_trace.py) host time of the hash drop-in's flush, by part:
// 0 whole deferred flushes, 1 waiting for a pool report, 2 prepare_batch, 3 kernel launches,
// 4 the call's end (k_free_unused), 5 flushes counted
static double g_host_us[8];
struct HostTimer {
    int slot;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit HostTimer(int s) : slot(s) {}
    ~HostTimer() {
        g_host_us[slot] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
};
#define TSDF_HOST_TIME(slot) HostTimer tsdf_host_timer_##slot(slot)
#else
#define TSDF_HOST_TIME(slot) ((void)0)
#endif

using namespace tsdf;

// A growable device array on the virtual-memory API: the address range for the largest size
// is reserved at create and physical chunks are mapped behind it as the pool grows.  Growth
// copies nothing and moves nothing, so launches already in flight (which only address blocks
// below their own max_blocks) keep running while it happens.  Falls back to hipMalloc + copy
// (grow_pool) when the reservation is refused.
struct VArray {
    char* base = nullptr;
    size_t reserved = 0, mapped = 0, gran = 0;
    int device = 0;
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
    hipMemAllocationProp prop() const {
        hipMemAllocationProp p{};
        p.type = hipMemAllocationTypePinned;
        p.location.type = hipMemLocationTypeDevice;
        p.location.id = device;
        return p;
    }
    bool reserve(int dev, size_t max_bytes) {  // false: VMM unavailable (use hipMalloc)
        device = dev;
        const hipMemAllocationProp p = prop();
        // the recommended granularity (the physical page the mapping is made of): chunks mapped at
        // offsets of the minimum granularity only were refused by hipMemMap
        if (hipMemGetAllocationGranularity(&gran, &p, hipMemAllocationGranularityRecommended) != hipSuccess || !gran) {
            (void)hipGetLastError();  // leave no sticky error behind
            return false;
        }
        piece = std::max(gran, kPiece / gran * gran);
        reserved = (max_bytes + piece - 1) / piece * piece;
        void* b = nullptr;
        if (hipMemAddressReserve(&b, reserved, std::max<size_t>(gran, 2u << 20), nullptr, 0) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        base = (char*)b;
        return true;
    }
    // Map [mapped, round_up(bytes)) in pieces of one size.  One size for every piece of an array:
    // on this ROCm a piece whose size differs from the one mapped before it is refused by
    // hipMemSetAccess ("invalid argument"), while equal pieces map at any count
    // (tools/gpu/vmm_probe.hip).  Pieces are only unmapped at release or to undo a failed growth
    // (pieces no kernel has used): an address range that kernels have written is never unmapped
    // and mapped again -- measured on the box, a piece mapped where a used one had been unmapped
    // lost the writes of one 2 MB fragment to a stale translation (tools/gpu/vmm_diag.py), so the
    // pool hands memory back by compaction into fresh ranges (trim_pool).
    static constexpr size_t kPiece = 8ull << 20;
    size_t piece = 0;
    int grow(size_t bytes) {
        const size_t want = (bytes + piece - 1) / piece * piece;
        if (want > reserved) return set_error(TSDF_E_CAPACITY, "pool beyond its reservation");
        while (mapped < want) TSDF_TRY(map_piece(piece));
        return TSDF_OK;
    }
    int map_piece(size_t sz) {
        const hipMemAllocationProp p = prop();
        hipMemGenericAllocationHandle_t hdl;
        hipError_t e = hipMemCreate(&hdl, sz, &p, 0);
        if (e == hipSuccess) {
            e = hipMemMap(base + mapped, sz, 0, hdl, 0);
            if (e == hipSuccess) {
                hipMemAccessDesc acc{};
                acc.location = p.location;
                acc.flags = hipMemAccessFlagsProtReadWrite;
                e = hipMemSetAccess(base + mapped, sz, &acc, 1);
                if (e != hipSuccess) (void)hipMemUnmap(base + mapped, sz);
            }
            if (e != hipSuccess) (void)hipMemRelease(hdl);
        }
        if (e != hipSuccess) {
            (void)hipGetLastError();  // no sticky error: the caller falls back to plain allocations
            return set_error(e == hipErrorOutOfMemory ? TSDF_E_OOM : TSDF_E_HIP, "pool mapping: %s",
                             hipGetErrorString(e));
        }
        chunks.emplace_back(hdl, sz);
        mapped += sz;
        return TSDF_OK;
    }
    // undo the mappings made after the array held `n_chunks` chunks (a failed multi-array growth)
    void unmap_to(size_t n_chunks) {
        while (chunks.size() > n_chunks) {
            const auto c = chunks.back();
            chunks.pop_back();
            mapped -= c.second;
            (void)hipMemUnmap(base + mapped, c.second);
            (void)hipMemRelease(c.first);
        }
    }
    // Unmap and release the physical memory.  The address range itself goes into `retired` when
    // kernels may have used it (kept reserved until the handle is destroyed, so no later reservation
    // -- a trim's or a growth's -- can be handed the same virtual addresses and map over a range
    // whose stale translations lost writes before, see above); with retired == nullptr (a range
    // no kernel has touched, or the handle's end) it is freed at once.
    void release(std::vector<std::pair<char*, size_t>>* retired = nullptr) {
        size_t off = mapped;
        for (auto it = chunks.rbegin(); it != chunks.rend(); ++it) {
            off -= it->second;
            (void)hipMemUnmap(base + off, it->second);
            (void)hipMemRelease(it->first);
        }
        chunks.clear();
        if (base) {
            if (retired) retired->emplace_back(base, reserved);
            else (void)hipMemAddressFree(base, reserved);
        }
        base = nullptr;
        mapped = reserved = 0;
    }
};

struct tsdf_hash {
    Base b;
    Table t{};          // device view (pointers + capacity)
    // The table size the API speaks of (map_size, hash_fusion.py:34-36): hash_function()'s modulus,
    // doubled by double_table_size and by the 0.75 load-factor policy.  The device table has
    // t.capacity = the next power of two >= map_size slots, so the home slot and the shard owner are
    // a mask and a shift in every kernel, whatever size the caller asked for (the reference's
    // default 10^6 and the demo's 2*10^6 included).
    long long map_size = 0;
    PoolState host_st{};
    ListEntry* d_list = nullptr;  // re-run list
    int list_cap = 0;
    int* d_res = nullptr;  // fused launches: per-brick claim words, one array per buffer set
    int* d_ins = nullptr;  // fused launches: bricks their culls inserted since the last k_free_unused
    // A deferred batch launched by the drop-in's per-frame calls (TSDF_DEFER) whose overflow check
    // waits for the next call on the handle (hash_settle): its frames and prepped buffers stay
    // untouched until then, so a skipped brick is still re-run exactly, before any later frame.
    struct Pending {
        bool on = false;
        Batch bt;
        int dk = 0, ck = 0;
        long long seq = -1;  // its integrate launch (the pool report the settle reads)
    } pend;
    // Fused calls rotate the buffer sets across calls (batch j of a call uses set (j + set_rot) %
    // kSets), so a deferred batch's prep / cull can be issued while the previous batch is still
    // pending: its buffers stay intact for an exact re-run.
    int set_rot = 0;
    bool fused = true;  // three-stage launches (k_fused_hash) when a call allows them
    // Asynchronous calls (TSDF_ASYNC): every allocating launch reports its pool state into
    // page-locked host memory (PoolReport, slot seq % kReports); before issuing launch s the host
    // reads launch s-2's report and grows the pool / table while there is still room for the
    // launches in flight, so no brick has to be skipped.  A skipped brick cannot be re-run
    // exactly later (its batch's frames are gone), so it is reported as TSDF_E_CAPACITY.
    PoolReport* h_rb = nullptr;   // host view of the report slots (hipHostMalloc, mapped)
    long long seq = 0;            // allocating launches issued so far
    long long rb_used = -1;       // live blocks in the last report read (or at the last sync check)
    long long deltas[4] = {};     // growth of live blocks over the last four reports / checks
    int n_delta = 0;
    void note_live(long long used) {  // a new live-block count: remember its growth (from 0 at first)
        const long long prev = rb_used < 0 ? 0 : rb_used;
        if (used != prev || rb_used < 0) deltas[n_delta++ & 3] = used > prev ? used - prev : 0;
        rb_used = used;
    }
    long long recent_growth() const {  // the largest of the recent growths (at least 256 blocks)
        return std::max<long long>({deltas[0], deltas[1], deltas[2], deltas[3], 256});
    }
    long long tomb_est = 0;       // PoolState::tombs at the last read or pool report (remove() and
                                  // k_free_unused add tombstones)
    // allocating launches issued before the table's last rebuild (resize_table drains the stream, so
    // every launch < rehash_seq had finished): their pool reports carry the tombstone count of the
    // table that was replaced and must not be read back into tomb_est (table_tombs)
    long long rehash_seq = 0;
    long long table_rebuilds = 0;  // rebuilds at the same size (tombstone purges), for the tests
    bool async_pending = false;   // asynchronous launches since the last overflow check
    // table load factor that triggers a doubling: the reference's hard-coded 0.75 (hash_fusion.py:
    // 156-161); TSDF_HASH_MAX_LOAD overrides it for the load-factor sweep (tools/hash_sweep.py)
    double max_load = 0.75;
    // block pool on reserved address ranges (tsdf, weight, colour, entry words, free list)
    bool vmm = false;
    VArray va[5];
    // address ranges of pool arrays that kernels used and that were since compacted away (trim) or
    // replaced by plain allocations: unmapped, but reserved until destroy (VArray::release)
    std::vector<std::pair<char*, size_t>> retired_va;
    int vmm_fail_at = -1;  // test hook (TSDF_HASH_VMM_FAIL=k): the next growth of array k fails
    bool async_grow = true;  // test hook (TSDF_HASH_ASYNC_GROW=0): asynchronous calls never grow ahead
    static constexpr size_t kPer[5] = {sizeof(float) * kBrickVox, sizeof(float) * kBrickVox, sizeof(float) * kBrickVox,
                                       sizeof(unsigned long long) * 8, sizeof(int)};
    long long mapped_blocks() const {  // blocks every pool array has memory for
        long long n = LLONG_MAX;
        for (int k = 0; k < 5; ++k) n = std::min<long long>(n, (long long)(va[k].mapped / kPer[k]));
        return n;
    }
    // Back blocks [0, n) of every pool array, all or nothing: if one array cannot grow, the
    // arrays grown before it are unmapped back to their old size, so the pool stays consistent
    // for the copy fallback (grow_pool).
    int map_pool(long long n) {
        const size_t per[5] = {sizeof(float) * kBrickVox, sizeof(float) * kBrickVox, sizeof(float) * kBrickVox,
                               sizeof(unsigned long long) * 8, sizeof(int)};
        size_t before[5];
        for (int k = 0; k < 5; ++k) before[k] = va[k].chunks.size();
        for (int k = 0; k < 5; ++k) {
            int r = TSDF_OK;
            if (k == vmm_fail_at) {
                vmm_fail_at = -1;
                r = set_error(TSDF_E_OOM, "pool mapping refused (test hook)");
            } else {
                r = va[k].grow(per[k] * (size_t)n);
            }
            if (r != TSDF_OK) {  // (array k may hold some of its new pieces too)
                for (int j = 0; j <= k; ++j) va[j].unmap_to(before[j]);
                return r;
            }
        }
        return TSDF_OK;
    }
};

namespace {

// Vol::canon over the allocated blocks after a set or an import (blocks past pool_top are
// initialised when they are handed out)
int recheck_canon(tsdf_hash* h) {
    PoolState st{};
    TSDF_HIP(hipMemcpyAsync(&st, h->t.st, sizeof(st), hipMemcpyDeviceToHost, h->b.stream));
    TSDF_HIP(hipStreamSynchronize(h->b.stream));
    return h->b.check_canon(st.pool_top * kBrickVox);
}

struct InfoDev {
    unsigned long long used, tomb, displaced, max_probe, entries;
};

// Empty slots hold value -1 (invariant: a slot's value is -1 whenever its key is empty or a
// tombstone), so a reader that sees a key inserted concurrently -- the CAS of the key comes before
// the store of its value -- reads -1, never a stale block (the fused hash launch's cull looks
// blocks up while the integrate of the batch before inserts: cull_lookup).
__global__ void k_fill_keys(unsigned long long* k, int* vals, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        k[i] = kEmpty;
        vals[i] = -1;
    }
}

// After each allocating launch: fold the launch's allocations into the pool state.
__global__ void k_commit(PoolState* st, long long max_blocks, PoolReport* rb, long long seq,
                         const unsigned* count) {
    commit_pool(st, max_blocks, rb, seq, count);
}

// Single-thread linear probe; returns the slot or -1.
__device__ long long probe_find(const Table& t, unsigned long long key, long long home) {
    long long s = home;
    for (long long n = 0; n < t.capacity; ++n) {
        const unsigned long long k = coh_load(&t.keys[s]);
        if (k == key) return s;
        if (k == kEmpty) return -1;
        if (++s == t.capacity) s = 0;
    }
    return -1;
}

__device__ bool voxel_brick(const Vol& v, long long x, long long y, long long z, int* bx, int* by,
                            int* bz, int* local) {
    if (x < 0 || y < 0 || z < 0 || x >= v.dims[0] || y >= v.dims[1] || z >= v.dims[2]) return false;
    *bx = (int)(x >> 3);
    *by = (int)(y >> 3);
    *bz = (int)(z >> 3);
    *local = (int)(((x & 7) * 8 + (y & 7)) * 8 + (z & 7));  // pool index; entry bit: word z, bit x*8+y
    return true;
}

__global__ void k_lookup(Vol v, Table t, Pool pool, const long long* ijk, long long n, float* ot,
                         float* ow, float* oc, unsigned char* found) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int bx, by, bz, local;
    unsigned char f = 0;
    float tv = 1.0f, wv = 0.0f, cv = 0.0f;
    if (voxel_brick(v, ijk[3 * i], ijk[3 * i + 1], ijk[3 * i + 2], &bx, &by, &bz, &local)) {
        const long long s = probe_find(t, pack_key(bx, by, bz), ref_hash(bx, by, bz, t.capacity, t.int_bits));
        if (s >= 0) {
            const long long blk = coh_load(&t.vals[s]);
            const unsigned long long word = coh_load(&t.occ[blk * 8 + (local & 7)]);
            if ((word >> (local >> 3)) & 1ull) {
                f = 1;
                const size_t j = (size_t)blk * kBrickVox + local;
                tv = coh_load(&pool.tsdf[j]);
                wv = coh_load(&pool.weight[j]);
                cv = coh_load(&pool.color[j]);
            }
        }
    }
    found[i] = f;
    if (ot) ot[i] = tv;
    if (ow) ow[i] = wv;
    if (oc) oc[i] = cv;
}

// Find-or-insert of unique block keys, one thread per key.  Keys are distinct, but two
// threads can race for the same empty slot: the loser keeps its block and probes on.  New
// blocks are initialised to (1, 0, 0) with empty entry masks.
__global__ void k_insert_blocks(Table t, Pool pool, const unsigned long long* keys, long long n,
                                int* blk_out, long long* slot_out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = keys[i];
    const int bx = (int)(key & 0x1FFFFF), by = (int)((key >> 21) & 0x1FFFFF), bz = (int)(key >> 42);
    long long s = ref_hash(bx, by, bz, t.capacity, t.int_bits);
    long long tomb = -1;
    int b = -1;
    blk_out[i] = -1;
    slot_out[i] = -1;
    for (long long m = 0; m < 2 * t.capacity; ++m) {
        const unsigned long long k = coh_load(&t.keys[s]);
        if (k == key) {
            blk_out[i] = coh_load(&t.vals[s]);
            slot_out[i] = s;
            return;  // (a spare block from a lost race stays unused)
        }
        if (k == kTomb && tomb < 0) tomb = s;
        if (k == kEmpty) {
            const long long target = tomb >= 0 ? tomb : s;
            const unsigned long long expect = tomb >= 0 ? kTomb : kEmpty;
            if (b < 0) b = pool_alloc(t);
            if (b < 0) return;  // pool full
            if (atomicCAS(&t.keys[target], expect, key) == expect) {
                coh_store(&t.vals[target], b);
                for (int k2 = 0; k2 < 8; ++k2) coh_store(&t.occ[(size_t)b * 8 + k2], 0ull);
                for (int j = 0; j < kBrickVox; ++j) {
                    pool.tsdf[(size_t)b * kBrickVox + j] = 1.0f;
                    pool.weight[(size_t)b * kBrickVox + j] = 0.0f;
                    pool.color[(size_t)b * kBrickVox + j] = 0.0f;
                }
                blk_out[i] = b;
                slot_out[i] = target;
                return;
            }
            // lost the slot to another key: probe on past it
            s = target;
            tomb = -1;
        }
        if (++s == t.capacity) s = 0;
    }
}

__global__ void k_set_voxels(Vol v, Table t, Pool pool, const long long* ijk, long long n,
                             const float* it, const float* iw, const float* ic) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int bx, by, bz, local;
    if (!voxel_brick(v, ijk[3 * i], ijk[3 * i + 1], ijk[3 * i + 2], &bx, &by, &bz, &local)) return;
    const long long s = probe_find(t, pack_key(bx, by, bz), ref_hash(bx, by, bz, t.capacity, t.int_bits));
    if (s < 0) return;
    const long long blk = coh_load(&t.vals[s]);
    atomicOr(&t.occ[blk * 8 + (local & 7)], 1ull << (local >> 3));
    const size_t j = (size_t)blk * kBrickVox + local;
    if (it) pool.tsdf[j] = it[i];
    if (iw) pool.weight[j] = iw[i];
    if (ic) pool.color[j] = ic[i];
}

__global__ void k_remove_voxels(Vol v, Table t, const long long* ijk, long long n,
                                unsigned char* removed) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int bx, by, bz, local;
    unsigned char r = 0;
    if (voxel_brick(v, ijk[3 * i], ijk[3 * i + 1], ijk[3 * i + 2], &bx, &by, &bz, &local)) {
        const long long s = probe_find(t, pack_key(bx, by, bz), ref_hash(bx, by, bz, t.capacity, t.int_bits));
        if (s >= 0) {
            const long long blk = coh_load(&t.vals[s]);
            const unsigned long long bit = 1ull << (local >> 3);
            const unsigned long long old = atomicAnd(&t.occ[blk * 8 + (local & 7)], ~bit);
            r = (old & bit) ? 1 : 0;
        }
    }
    if (removed) removed[i] = r;
}

// Blocks whose every entry is gone are unlinked (tombstone) and returned to the free list.
__global__ void k_free_empty(Table t, const unsigned long long* keys, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = keys[i];
    const int bx = (int)(key & 0x1FFFFF), by = (int)((key >> 21) & 0x1FFFFF), bz = (int)(key >> 42);
    const long long s = probe_find(t, key, ref_hash(bx, by, bz, t.capacity, t.int_bits));
    if (s < 0) return;
    const long long blk = coh_load(&t.vals[s]);
    for (int k = 0; k < 8; ++k)
        if (coh_load(&t.occ[blk * 8 + k])) return;
    coh_store(&t.vals[s], -1);  // (the empty-slot invariant, k_fill_keys)
    coh_store(&t.keys[s], kTomb);
    atomicAdd((unsigned long long*)&t.st->tombs, 1ull);
    const unsigned long long f = atomicAdd((unsigned long long*)&t.st->free_count, 1ull);
    coh_store(&t.free_list[f], (int)blk);
}

// The end of a fused call: the blocks its culls inserted (Table::ins_list) that no frame gave an
// entry are unlinked and returned to the free list, so the table holds exactly the reference's
// keys.  A freed slot whose successor is empty becomes empty again (no probe passes through it to a
// later key); otherwise a tombstone.  Nothing else runs on the table meanwhile (stream order: after
// the call's last launch, which has no cull).
__global__ void k_free_unused(Vol v, Table t) {
    const long long n = min(coh_load(&t.st->n_inserted), t.ins_cap);
    const int nb12 = v.nb[1] * v.nb[2];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const int e = t.ins_list[i];
        if (e < 0) {  // a spare block of a probe that ran out of slots (spare_block): back to the free list
            const unsigned long long f = atomicAdd((unsigned long long*)&t.st->free_count, 1ull);
            coh_store(&t.free_list[f], -2 - e);
            continue;
        }
        const int bx = e / nb12, r = e - bx * nb12, by = r / v.nb[2], bz = r - by * v.nb[2];
        const long long s = probe_find(t, pack_key(bx, by, bz), ref_hash(bx, by, bz, t.capacity, t.int_bits));
        if (s < 0) continue;
        const int blk = coh_load(&t.vals[s]);
        bool used = false;
        for (int k = 0; k < 8; ++k) used |= coh_load(&t.occ[(size_t)blk * 8 + k]) != 0ull;
        if (used) continue;
        const long long nx = s + 1 == t.capacity ? 0 : s + 1;
        const bool last = coh_load(&t.keys[nx]) == kEmpty;
        coh_store(&t.vals[s], -1);  // (the empty-slot invariant, k_fill_keys)
        coh_store(&t.keys[s], last ? kEmpty : kTomb);
        if (!last) atomicAdd((unsigned long long*)&t.st->tombs, 1ull);
        const unsigned long long f = atomicAdd((unsigned long long*)&t.st->free_count, 1ull);
        coh_store(&t.free_list[f], blk);
    }
}

__global__ void k_rehash(Table src, Table dst) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < src.capacity;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long key = coh_load(&src.keys[i]);
        if (key == kEmpty || key == kTomb) continue;
        const int bx = (int)(key & 0x1FFFFF), by = (int)((key >> 21) & 0x1FFFFF), bz = (int)(key >> 42);
        long long s = ref_hash(bx, by, bz, dst.capacity, dst.int_bits);
        for (long long m = 0; m < dst.capacity; ++m) {
            if (atomicCAS(&dst.keys[s], kEmpty, key) == kEmpty) {
                coh_store(&dst.vals[s], coh_load(&src.vals[i]));
                break;
            }
            if (++s == dst.capacity) s = 0;
        }
    }
}

__global__ void k_info(Table t, InfoDev* out) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < t.capacity;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long key = coh_load(&t.keys[i]);
        if (key == kEmpty) continue;
        if (key == kTomb) {
            atomicAdd(&out->tomb, 1ull);
            continue;
        }
        atomicAdd(&out->used, 1ull);
        const int bx = (int)(key & 0x1FFFFF), by = (int)((key >> 21) & 0x1FFFFF), bz = (int)(key >> 42);
        const long long home = ref_hash(bx, by, bz, t.capacity, t.int_bits);
        const long long d = (i - home + t.capacity) % t.capacity;
        if (d) atomicAdd(&out->displaced, 1ull);
        atomicMax(&out->max_probe, (unsigned long long)d);
        const long long blk = coh_load(&t.vals[i]);
        unsigned long long c = 0;
        for (int k = 0; k < 8; ++k) c += __popcll(coh_load(&t.occ[blk * 8 + k]));
        if (c) atomicAdd(&out->entries, c);
    }
}

// Densify into a dense handle's brick pool (same dims, so brick b of block (bx,by,bz) is
// (bx*nb1 + by)*nb2 + bz with the same voxel order inside): one thread per (slot, z-plane of the
// block); the voxels with an entry are copied, the others keep the dense handle's (1, 0, 0).
__global__ void k_to_bricks(Vol v, Table t, Pool pool, Pool dst) {
    const long long total = t.capacity * kBrickEdge;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long s = i >> 3;
        const int kz = (int)(i & 7);
        const unsigned long long key = coh_load(&t.keys[s]);
        if (key == kEmpty || key == kTomb) continue;
        const long long blk = coh_load(&t.vals[s]);
        unsigned long long m = coh_load(&t.occ[blk * 8 + kz]);
        const long long bx = (long long)(key & 0x1FFFFF), by = (long long)((key >> 21) & 0x1FFFFF),
                        bz = (long long)(key >> 42);
        const size_t b = (size_t)((bx * v.nb[1] + by) * v.nb[2] + bz);
        while (m) {
            const int bit = __ffsll((long long)m) - 1;
            m &= m - 1;
            const size_t o = b * kBrickVox + bit * 8 + kz;
            const size_t j = (size_t)blk * kBrickVox + bit * 8 + kz;
            dst.tsdf[o] = coh_load(&pool.tsdf[j]);
            dst.weight[o] = coh_load(&pool.weight[j]);
            dst.color[o] = coh_load(&pool.color[j]);
        }
    }
}

// Densify (hash_fusion.py:442-463): one thread per (slot, z-plane of the block); the 64 bits
// of that plane's entry mask select the voxels to write.
__global__ void k_to_dense(Vol v, Table t, Pool pool, float* ot, float* ow, float* oc) {
    const long long total = t.capacity * kBrickEdge;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long s = i >> 3;
        const int kz = (int)(i & 7);
        const unsigned long long key = coh_load(&t.keys[s]);
        if (key == kEmpty || key == kTomb) continue;
        const long long blk = coh_load(&t.vals[s]);
        unsigned long long m = coh_load(&t.occ[blk * 8 + kz]);
        const int bx = (int)(key & 0x1FFFFF), by = (int)((key >> 21) & 0x1FFFFF), bz = (int)(key >> 42);
        while (m) {
            const int bit = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int x = bx * 8 + (bit >> 3), y = by * 8 + (bit & 7), z = bz * 8 + kz;
            if (x >= v.dims[0] || y >= v.dims[1] || z >= v.dims[2]) continue;
            const size_t o = ((size_t)x * v.dims[1] + y) * v.dims[2] + z;
            const size_t j = (size_t)blk * kBrickVox + bit * 8 + kz;
            if (ot) ot[o] = coh_load(&pool.tsdf[j]);
            if (ow) ow[o] = coh_load(&pool.weight[j]);
            if (oc) oc[o] = coh_load(&pool.color[j]);
        }
    }
}

// Live blocks out (one wave per slot): block coordinates, the 512 voxels of each field in the
// brick-local order (x*8 + y)*8 + z, and the 8 entry words.  Output order = claim order.
__global__ void k_export_blocks(Table t, Pool pool, unsigned long long* counter, long long cap, int* bxyz,
                                float* ot, float* ow, float* oc, unsigned long long* oocc) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long s = wave; s < t.capacity; s += nw) {
        const unsigned long long key = coh_load(&t.keys[s]);
        if (key == kEmpty || key == kTomb) continue;
        long long i = 0;
        if (lane == 0) i = (long long)atomicAdd(counter, 1ull);
        i = __shfl(i, 0);
        if (i >= cap) continue;
        const long long blk = coh_load(&t.vals[s]);
        if (lane < 3) bxyz[3 * i + lane] = (int)((key >> (21 * lane)) & 0x1FFFFF);
        if (lane < 8 && oocc) oocc[8 * i + lane] = coh_load(&t.occ[blk * 8 + lane]);
        const size_t src = (size_t)blk * kBrickVox + (size_t)lane * 8, dst = (size_t)i * kBrickVox + (size_t)lane * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (ot) *(float4*)(ot + dst + 4 * h) = *(const float4*)(pool.tsdf + src + 4 * h);
            if (ow) *(float4*)(ow + dst + 4 * h) = *(const float4*)(pool.weight + src + 4 * h);
            if (oc) *(float4*)(oc + dst + 4 * h) = *(const float4*)(pool.color + src + 4 * h);
        }
    }
}

// Imported blocks in (one wave per block; blk from k_insert_blocks): contents and entry words
// overwrite the block.
__global__ void k_write_blocks(Table t, Pool pool, const int* blk, long long n, const float* it, const float* iw,
                               const float* ic, const unsigned long long* iocc) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long i = wave; i < n; i += nw) {
        const long long b = blk[i];
        if (b < 0) continue;
        if (lane < 8) coh_store(&t.occ[b * 8 + lane], iocc ? iocc[8 * i + lane] : ~0ull);
        const size_t dst = (size_t)b * kBrickVox + (size_t)lane * 8, src = (size_t)i * kBrickVox + (size_t)lane * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (it) *(float4*)(pool.tsdf + dst + 4 * h) = *(const float4*)(it + src + 4 * h);
            if (iw) *(float4*)(pool.weight + dst + 4 * h) = *(const float4*)(iw + src + 4 * h);
            if (ic) *(float4*)(pool.color + dst + 4 * h) = *(const float4*)(ic + src + 4 * h);
        }
    }
}

__global__ void k_fill_dense(float* t, float* w, float* c, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        if (t) t[i] = 1.0f;
        if (w) w[i] = 0.0f;
        if (c) c[i] = 0.0f;
    }
}

// Device buffers freed on every exit path unless keep() is called (the error paths of a
// multi-buffer allocation free what was already allocated).
struct DevBufs {
    std::vector<void*> p;
    ~DevBufs() {
        for (void* q : p)
            if (q) (void)hipFree(q);
    }
    void* add(void* q) {
        p.push_back(q);
        return q;
    }
    void keep() { p.clear(); }
};

template <typename T>
int dev_alloc(DevBufs& bufs, T** out, size_t bytes) {
    *out = nullptr;
    TSDF_HIP(hipMalloc((void**)out, bytes));
    bufs.add(*out);
    return TSDF_OK;
}

int read_state(tsdf_hash* h) {
    TSDF_HIP(hipMemcpyAsync(&h->host_st, h->t.st, sizeof(PoolState), hipMemcpyDeviceToHost, h->b.stream));
    TSDF_HIP(hipStreamSynchronize(h->b.stream));
    h->tomb_est = h->host_st.tombs;
    return TSDF_OK;
}

// The size the pool grows to when it needs room for `need` blocks.  Mapped chunks (VMM) cost no
// copy and no drain, so the pool follows the live blocks closely: 1/16 over the need, which the
// callers size as the live blocks plus the growth of the batches in flight; the copy path
// doubles (each growth copies the whole pool).
long long pool_target(const tsdf_hash* h, long long need) {
    if (!h->vmm) return std::max(h->t.max_blocks * 2, need);
    return std::max(h->t.max_blocks, need + need / 16);
}

int grow_pool(tsdf_hash* h, long long new_max) {
    Base& B = h->b;
    Table& t = h->t;
    // the volume has n_bricks bricks: a pool never needs more blocks than that
    new_max = std::min<long long>(new_max, B.n_bricks);
    if (new_max <= t.max_blocks) return TSDF_OK;
    if (h->vmm) {  // map more physical memory behind the reserved ranges: no copy, no drain
        if (h->map_pool(new_max) == TSDF_OK) {
            t.max_blocks = std::min<long long>(h->mapped_blocks(), B.n_bricks);  // (whole pieces)
            return TSDF_OK;
        }
        // mapping refused: continue with plain allocations (copy below, then unmap the ranges)
    }
    const size_t old_n = (size_t)t.max_blocks, nn = (size_t)new_max;
    float *nt, *nw, *nc;
    unsigned long long* no;
    int* nf;
    TSDF_HIP(hipStreamSynchronize(B.stream));
    DevBufs fresh;  // freed again if any allocation or copy fails
    TSDF_TRY(dev_alloc(fresh, &nt, nn * kBrickVox * sizeof(float)));
    TSDF_TRY(dev_alloc(fresh, &nw, nn * kBrickVox * sizeof(float)));
    TSDF_TRY(dev_alloc(fresh, &nc, nn * kBrickVox * sizeof(float)));
    TSDF_TRY(dev_alloc(fresh, &no, nn * 8 * sizeof(unsigned long long)));
    TSDF_TRY(dev_alloc(fresh, &nf, nn * sizeof(int)));
    TSDF_HIP(hipMemcpyAsync(nt, B.pool.tsdf, old_n * kBrickVox * sizeof(float), hipMemcpyDeviceToDevice, B.stream));
    TSDF_HIP(hipMemcpyAsync(nw, B.pool.weight, old_n * kBrickVox * sizeof(float), hipMemcpyDeviceToDevice, B.stream));
    TSDF_HIP(hipMemcpyAsync(nc, B.pool.color, old_n * kBrickVox * sizeof(float), hipMemcpyDeviceToDevice, B.stream));
    TSDF_HIP(hipMemcpyAsync(no, t.occ, old_n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, B.stream));
    TSDF_HIP(hipMemcpyAsync(nf, t.free_list, old_n * sizeof(int), hipMemcpyDeviceToDevice, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    fresh.keep();
    if (h->vmm) {
        for (auto& v : h->va) v.release(&h->retired_va);
        h->vmm = false;
    } else {
        (void)hipFree(B.pool.tsdf);
        (void)hipFree(B.pool.weight);
        (void)hipFree(B.pool.color);
        (void)hipFree(t.occ);
        (void)hipFree(t.free_list);
    }
    B.pool.tsdf = nt;
    B.pool.weight = nw;
    B.pool.color = nc;
    t.occ = no;
    t.free_list = nf;
    t.max_blocks = new_max;
    return TSDF_OK;
}

// Hand mapped pool memory above the bump pointer back (VMM pools only, at a sync point: nothing is
// in flight): the blocks [0, pool_top) and the free list move into fresh reserved ranges mapped for
// pool_top + 1/32 of it (at least 256 blocks), rounded up to whole pieces, and the old ranges are
// released -- so after an asynchronous run, whose growth had to stay ahead of the launches in
// flight, the pool holds about the live blocks again.  A compaction, not an unmap of the top
// pieces: see VArray::grow.  One device copy of the live state (~1.1 GB at 512^3: ~0.5 ms).
// Nothing changes when the new ranges cannot be had.
int trim_pool(tsdf_hash* h) {
    if (!h->vmm) return TSDF_OK;
    TSDF_TRY(read_state(h));
    const long long top = h->host_st.pool_top;
    const long long keep = std::max<long long>(top + std::max<long long>(256, top / 32), 64);
    if (keep + (long long)(VArray::kPiece / tsdf_hash::kPer[0]) > h->t.max_blocks) return TSDF_OK;  // < one piece to gain
    const size_t nb = (size_t)h->b.n_bricks;
    VArray nv[5];
    bool ok = true;
    for (int k = 0; k < 5 && ok; ++k)
        ok = nv[k].reserve(h->b.device, tsdf_hash::kPer[k] * nb) && nv[k].grow(tsdf_hash::kPer[k] * (size_t)keep) == TSDF_OK;
    if (ok) {
        const long long n = std::min<long long>(keep, h->t.max_blocks);  // (>= pool_top, >= free_count)
        for (int k = 0; k < 5 && ok; ++k)
            ok = hipMemcpyAsync(nv[k].base, h->va[k].base, tsdf_hash::kPer[k] * (size_t)n, hipMemcpyDeviceToDevice,
                                h->b.stream) == hipSuccess;
        ok = ok && hipStreamSynchronize(h->b.stream) == hipSuccess;
    }
    if (!ok) {  // keep the pool as it is (copies may have written the new ranges: retire them too)
        (void)hipGetLastError();
        for (auto& v : nv) v.release(&h->retired_va);
        return TSDF_OK;
    }
    for (int k = 0; k < 5; ++k) {
        h->va[k].release(&h->retired_va);
        h->va[k] = nv[k];
        nv[k] = VArray{};
    }
    h->b.pool.tsdf = (float*)h->va[0].base;
    h->b.pool.weight = (float*)h->va[1].base;
    h->b.pool.color = (float*)h->va[2].base;
    h->t.occ = (unsigned long long*)h->va[3].base;
    h->t.free_list = (int*)h->va[4].base;
    h->t.max_blocks = std::min<long long>(h->mapped_blocks(), h->b.n_bricks);
    return TSDF_OK;
}

int resize_table(tsdf_hash* h, long long new_cap) {
    Base& B = h->b;
    Table nt = h->t;
    nt.capacity = new_cap;
    DevBufs fresh;
    TSDF_TRY(dev_alloc(fresh, &nt.keys, sizeof(unsigned long long) * new_cap));
    TSDF_TRY(dev_alloc(fresh, &nt.vals, sizeof(int) * new_cap));
    hipLaunchKernelGGL(k_fill_keys, dim3(2048), dim3(256), 0, B.stream, nt.keys, nt.vals, (long long)new_cap);
    TSDF_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_rehash, dim3(2048), dim3(256), 0, B.stream, h->t, nt);
    TSDF_HIP(hipGetLastError());
    TSDF_HIP(hipMemsetAsync(&h->t.st->tombs, 0, sizeof(long long), B.stream));  // a rebuilt table has none
    TSDF_HIP(hipStreamSynchronize(B.stream));
    fresh.keep();
    h->tomb_est = 0;
    h->host_st.tombs = 0;
    h->rehash_seq = h->seq;
    (void)hipFree(h->t.keys);
    (void)hipFree(h->t.vals);
    h->t.keys = nt.keys;
    h->t.vals = nt.vals;
    h->t.capacity = new_cap;
    return TSDF_OK;
}

long long next_pow2(long long n) {
    long long p = 1;
    while (p < n) p <<= 1;
    return p;
}

// The tombstone count of a pool report of launch `seq`, or 0 when that launch ran on a table that
// has since been rebuilt (rehash_seq): the rebuild cleared those tombstones.  Round 5 took the max
// of the estimate and every report, so a report written just before a rebuild brought the old
// count back and the policy below counted tombstones the table no longer had.
long long table_tombs(const tsdf_hash* h, long long seq, long long report_tombs) {
    return seq < h->rehash_seq ? h->tomb_est : std::max(h->tomb_est, report_tombs);
}

// Room in the table for `live` keys plus `extra` new ones, keeping the reference's policy
// (needs_resize / double_table_size, hash_fusion.py:156-161,414-437): the table size doubles while
// live + extra keys reach max_load of it -- it grows with its keys, as the reference's does, never
// with deletions; tombstones (k_free_unused, remove) count against the slots but only make the
// table rebuild at its size (a purge), so a long per-frame run whose calls free their unused
// blocks does not double the table (round 5 doubled for them).  The doublings are computed first
// and done as ONE rehash; `slots_room` > 0 also keeps live + extra + tombstones below 31/32 of
// the device slots (asynchronous calls: room for the launches in flight, whatever the policy).
// Live keys are bricks of the volume, so extra is clamped to the bricks not yet keyed and the
// sizes asked are bounded by 2 * n_bricks / max_load; a count outside that is a wrong estimate
// and fails with TSDF_E_CAPACITY instead of doubling until the device runs out of memory (round
// 5's OOM).
int table_room(tsdf_hash* h, long long live, long long extra, long long tombs, bool slots_room = false) {
    const long long nb = h->b.n_bricks;
    if (live < 0 || live > nb || tombs < 0)
        return set_error(TSDF_E_CAPACITY, "hash table: implausible counts (%lld live keys, %lld tombstones) for %lld "
                         "bricks and %lld slots", live, tombs, nb, (long long)h->t.capacity);
    // (the tombstone count is an upper bound -- it counts key -> tombstone transitions since the
    // last rebuild, and a slot can take several -- but no more slots than the table has)
    tombs = std::min<long long>(tombs, h->t.capacity);
    extra = std::max<long long>(0, std::min<long long>(extra, nb - live));
    const long long bound = std::max<long long>(h->map_size, (long long)(2.0 * (double)nb / h->max_load) + 64);
    long long ms = h->map_size;
    const auto slots_full = [&](long long m, long long t) {
        const long long cap = next_pow2(m);
        return slots_room && live + extra + t >= cap - cap / 32;
    };
    while ((double)(live + extra) >= h->max_load * (double)ms || slots_full(ms, 0)) {
        ms *= 2;
        if (ms > bound)
            return set_error(TSDF_E_CAPACITY, "hash table: %lld live keys + %lld of room would need a table of more "
                             "than %lld (max_load %.2f, %lld bricks)", live, extra, bound, h->max_load, nb);
    }
    if (ms != h->map_size) {  // one rehash to the policy's size (it drops the tombstones too)
        TSDF_TRY(resize_table(h, next_pow2(ms)));
        h->map_size = ms;
        return TSDF_OK;
    }
    if ((double)(live + extra + tombs) >= h->max_load * (double)ms || slots_full(ms, tombs)) {
        TSDF_TRY(resize_table(h, h->t.capacity));  // the purge: same size, no tombstones
        ++h->table_rebuilds;
    }
    return TSDF_OK;
}

int info_raw(tsdf_hash* h, InfoDev* out) {
    Base& B = h->b;
    InfoDev* d = nullptr;
    TSDF_HIP(hipMalloc(&d, sizeof(InfoDev)));
    TSDF_HIP(hipMemsetAsync(d, 0, sizeof(InfoDev), B.stream));
    hipLaunchKernelGGL(k_info, dim3(2048), dim3(256), 0, B.stream, h->t, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(InfoDev), hipMemcpyDeviceToHost, B.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(B.stream);
    (void)hipFree(d);
    TSDF_HIP(e);
    return TSDF_OK;
}

// Grow whatever ran out (reference policy: keep the keys below 0.75 of the table size, like
// needs_resize, hash_fusion.py:156-161), then re-run the bricks that were skipped.
// Live keys = blocks handed out and not freed; tombstones are bounded by PoolState::tombs -- no
// table scan per batch (k_info over 2^22 slots cost 1.5 ms).
int ensure_room(tsdf_hash* h, bool fresh = false) {
    if (!fresh) TSDF_TRY(read_state(h));  // fresh: host_st was read after the stream's last launch
    const long long live = h->host_st.pool_top - h->host_st.free_count;
    h->note_live(live);
    // the block pool keeps room for the next batches' growth: with mapped chunks about two
    // batches' worth over the live blocks (a batch that still runs out is re-run exactly after
    // growing, hash_after_batch); the copy path keeps the live blocks below 0.75 of the pool
    const long long step = h->recent_growth();
    if (h->vmm ? live + 2 * step > h->t.max_blocks : (double)(live + 64) >= 0.75 * (double)h->t.max_blocks)
        TSDF_TRY(grow_pool(h, pool_target(h, live + 3 * step)));
    return table_room(h, live, 0, h->host_st.tombs);
}

// Bricks skipped by asynchronous launches: their batches' frames are gone, so they cannot be
// re-run exactly; report them (once) and clear the overflow list so that no later synchronous
// call replays them against its own frames.
int take_overflow(tsdf_hash* h) {
    Base& B = h->b;
    TSDF_HIP(hipStreamSynchronize(B.stream));
    TSDF_TRY(read_state(h));
    h->async_pending = false;
    const long long n = h->host_st.n_overflow;
    if (n <= 0) return TSDF_OK;
    TSDF_HIP(hipMemsetAsync(&h->t.st->n_overflow, 0, sizeof(long long), B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    h->host_st.n_overflow = 0;
    return set_error(TSDF_E_CAPACITY,
                     "asynchronous hash integrate skipped %lld brick updates: the block pool (%lld) or table "
                     "(%lld slots) filled faster than it could grow; use synchronous calls or a larger "
                     "max_blocks / capacity",
                     n, (long long)h->t.max_blocks, (long long)h->t.capacity);
}

// Report of allocating launch s (written by its committing thread; waits for it).
int wait_report(tsdf_hash* h, long long s, PoolReport* out) {
    TSDF_HOST_TIME(1);
    volatile PoolReport* r = h->h_rb + (s % kReports);
    for (int spin = 0;; ++spin) {
        if (__atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) == s + 1) break;
        if (spin > 64) {
            const hipError_t q = hipStreamQuery(h->b.stream);
            if (q == hipSuccess && __atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) != s + 1)
                return set_error(TSDF_E_HIP, "pool report %lld missing after the stream drained", s);
            if (q != hipSuccess && q != hipErrorNotReady) TSDF_HIP(q);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    out->pool_top = r->pool_top;
    out->free_count = r->free_count;
    out->n_overflow = r->n_overflow;
    out->listed = r->listed;
    out->tombs = r->tombs;
    out->seq = s + 1;
    return TSDF_OK;
}

// Asynchronous calls, before issuing allocating launch s: launches s-1 and s may allocate before
// the next check.  Each can allocate at most the bricks its cull lists, and a batch's list is
// about as long as the one before it (the camera moves a little per batch), so the room kept is
// two of launch s-2's lists -- a bound that holds when the camera turns from a region it has
// mapped to one it has not (growth jumps from ~0 to the whole list), where the recent growth
// alone would not -- or three recent growths when larger.
int async_room(tsdf_hash* h, long long s) {
    if (s < 2) return TSDF_OK;
    PoolReport r;
    TSDF_TRY(wait_report(h, s - 2, &r));
    if (r.n_overflow > 0) return take_overflow(h);
    if (!h->async_grow) return TSDF_OK;
    const long long used = r.pool_top - r.free_count;
    h->note_live(used);
    h->tomb_est = table_tombs(h, s - 2, r.tombs);
    // (the copy path keeps the pool's 1/12 as a floor of the estimate too, and doubles)
    const long long step = h->vmm ? h->recent_growth() : std::max<long long>(h->recent_growth(), h->t.max_blocks / 12);
    const long long need = used + std::max<long long>(3 * step, 2 * r.listed + step);
    if (need > h->t.max_blocks) TSDF_TRY(grow_pool(h, pool_target(h, need + step)));
    TSDF_TRY(table_room(h, used, 3 * h->recent_growth(), h->tomb_est));
    // ... and the table's slots, whatever the load-factor policy allows (TSDF_HASH_MAX_LOAD up to
    // 0.99, or a jump in growth just below 0.75): the same two lists' worth of new keys must fit
    // below 31/32 of the slots, or launch s could find the table full and skip bricks
    const long long burst = std::max<long long>(3 * h->recent_growth(), 2 * r.listed + h->recent_growth());
    return table_room(h, used, burst, h->tomb_est, true);
}

// One hash integrate pass over a batch: the listed bricks (list/count from k_cull, or an
// explicit list of skipped entries).
void launch_integrate(tsdf_hash* h, const Batch& bt, int dk, int ck, const ListEntry* list,
                      unsigned int* count, int n_list) {
    Base& B = h->b;
    const unsigned grid = B.grid_for((const void*)k_integrate<true, 0, 0, true>);
    // (a batch of the fused path may carry texels: its re-run gathers them too)
    const int sel = bt.texel ? 4 : (dk == TSDF_DEPTH_U16_MM ? 0 : 2) | (ck == TSDF_COLOR_RGB8 ? 0 : 1);
    switch (sel) {
#define TSDF_LAUNCH(S, DK_, CK_)                                                                        \
    case S:                                                                                             \
        hipLaunchKernelGGL((k_integrate<true, DK_, CK_, true>), dim3(grid), dim3(kWG), 0, B.stream, B.vol, bt, \
                           B.pool, h->t, B.stats, list, count, n_list);                                 \
        break;
        TSDF_LAUNCH(0, 0, 0)
        TSDF_LAUNCH(1, 0, 1)
        TSDF_LAUNCH(2, 1, 0)
        TSDF_LAUNCH(3, 1, 1)
        TSDF_LAUNCH(4, 2, 0)
#undef TSDF_LAUNCH
    }
}

// Synchronous calls: recover from a full table/pool exactly (the skipped bricks of batch `bt`
// were not touched by any of its frames), then keep the reference's load-factor policy.
int hash_after_batch(tsdf_hash* h, const Batch& bt, int dk, int ck) {
    Base& B = h->b;
    TSDF_TRY(read_state(h));
    for (int round = 0; h->host_st.n_overflow > 0 && round < 40; ++round) {
        const long long n_ov = h->host_st.n_overflow;
        if (n_ov > h->t.overflow_cap)
            return set_error(TSDF_E_CAPACITY, "overflow list exceeded (%lld bricks)", n_ov);
        if (h->list_cap < n_ov) {
            if (h->d_list) (void)hipFree(h->d_list);
            TSDF_HIP(hipMalloc(&h->d_list, sizeof(ListEntry) * n_ov));
            h->list_cap = (int)n_ov;
        }
        TSDF_HIP(hipMemcpyAsync(h->d_list, h->t.overflow, sizeof(ListEntry) * n_ov, hipMemcpyDeviceToDevice, B.stream));
        TSDF_HIP(hipMemsetAsync(&h->t.st->n_overflow, 0, sizeof(long long), B.stream));
        // Grow what ran short.  A brick is skipped when its block found no slot (the table) or no
        // pool block; the fused cull of batch L ran in launch L-1 with the pool limit of then, so
        // after the previous batch's check grew the pool its skips find room now and need no
        // growth -- round 5 charged them to the table and doubled it for every such batch (the
        // sweep's fresh 2^22-slot tables hit table_room's bound on it).  A re-run
        // that still skips grows the pool past its limit.
        const long long live = h->host_st.pool_top - h->host_st.free_count;
        const bool pool_short = h->host_st.pool_top + n_ov > h->t.max_blocks - h->host_st.free_count;
        const bool table_short = live + h->host_st.tombs + n_ov >= h->t.capacity - h->t.capacity / 32;
        if (pool_short || (round > 0 && !table_short))
            TSDF_TRY(grow_pool(h, pool_target(h, std::max<long long>(h->host_st.pool_top + 2 * n_ov,
                                                                       h->t.max_blocks + n_ov))));
        if (table_short) TSDF_TRY(table_room(h, live, n_ov, h->host_st.tombs, true));
        launch_integrate(h, bt, dk, ck, h->d_list, nullptr, (int)n_ov);
        TSDF_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, B.stream, h->t.st, (long long)h->t.max_blocks,
                           (PoolReport*)nullptr, -1ll, (const unsigned*)nullptr);
        TSDF_HIP(hipGetLastError());
        TSDF_TRY(read_state(h));
    }
    if (h->host_st.n_overflow > 0) return set_error(TSDF_E_CAPACITY, "could not make room in the hash table");
    return TSDF_OK;
}

// Three-stage launches (k_fused_hash; the dense path's scheme, tsdf_dense.hip): launch L
// integrates batch L, culls L+1 -- finding or inserting its blocks into the claim words res_c --
// and preps L+2.  Synchronous calls check batch L's overflow before launch L+1 is issued; its
// re-run reads batch L's frames, which no launch has replaced.
// Invariant: block ids stay fixed between the cull that writes a claim word and the integrate that
// reads it.  What the host may run in between keeps them: a table resize rehashes keys, never values;
// grow_pool maps or copies blocks in place; an overflow re-run only updates or inserts blocks, and
// the integrate loads every block it is given (a block the cull inserted may have been updated by
// that re-run).  A future step that renumbers blocks between launches must rerun the cull.  Blocks
// are freed only after a call's last launch (k_free_unused), when no claim word is pending.
// Internal flag of hash_run: a synchronous call of at most one batch whose overflow check
// (hash_after_batch + ensure_room) is left to the next call on the handle (hash_settle).
constexpr int kCheckLater = 1 << 30;
int hash_settle(tsdf_hash* h);

int hash_run_fused(tsdf_hash* h, int n_frames, const void* depth, int dk, const void* color, int H, int W,
                   const double* K, const double* Tinv, int flags) {
    Base& B = h->b;
    const bool sync = !(flags & TSDF_ASYNC);
    const int nbat = B.batch;
    const bool later = sync && (flags & kCheckLater) && n_frames <= nbat;
    // a pending batch's exact re-run reads its buffer set and staging slot: settle it first if this
    // call reallocates per-batch buffers (first fused call, another image size)
    if (h->pend.on && !(B.n_sets >= kSets && B.pyr_H == H && B.pyr_W == W && B.stage_fits(dk, TSDF_COLOR_RGB8, H, W)))
        TSDF_TRY(hash_settle(h));
    TSDF_TRY(B.use_sets(kSets));
    const int rot = h->set_rot;
    const auto set_of = [rot](int j) { return (j + rot) % kSets; };
    const int nb = (n_frames + nbat - 1) / nbat;
    // a pending deferred batch uses one buffer set, which the loop's prep of batch 2 would reuse
    // (its exact re-run reads it): settle it before a call of several batches (round-4 advisor)
    if (h->pend.on && nb > 1) TSDF_TRY(hash_settle(h));
    if (!h->d_res) {  // each word is written by the cull that lists its brick before an integrate reads it
        if (B.n_bricks >= (1ll << 31) / kSets) return set_error(TSDF_E_ARG, "volume too large for the claim words");
        TSDF_HIP(hipMalloc(&h->d_res, sizeof(int) * kSets * (size_t)B.n_bricks));
        // the bricks the culls insert between two k_free_unused: distinct, so at most every brick
        TSDF_HIP(hipMalloc(&h->d_ins, sizeof(int) * (size_t)B.n_bricks));
        h->t.ins_list = h->d_ins;
        h->t.ins_cap = B.n_bricks;
    }
    const int gi_full = (int)B.grid_for((const void*)k_fused_hash<0>, kFusedHashWG);
    // (a shard that owns no brick -- more shards than bricks -- still runs one cull workgroup, which
    // lists nothing, like the in-line path's max(1, ...))
    const int gc_full = h->t.owned ? std::max(1, (h->t.n_owned + 63) / 64) : (int)B.cull_grid_fused();
    // texels (Base::texel_for) by the bricks this handle owns
    const bool tex = B.texel_for(dk, h->t.owned ? (long long)h->t.n_owned : B.n_bricks, Base::kTexelMinBricksHash);
    struct TexelScope {
        Base& b;
        ~TexelScope() { b.texel_now = false; }
    } tex_scope{B};
    B.texel_now = tex;
    Batch bts[kSets];
    h->set_rot = (rot + nb) % kSets;
    for (int L = -2; L < nb; ++L) {
        const int jp = L + 2;
        if (jp < nb) {
            const int f0 = jp * nbat;
            const int n = n_frames - f0 < nbat ? n_frames - f0 : nbat;
            B.use_set(set_of(jp));
            // HashTable.integrate ignores obs_weight (hash_fusion.py:141,145): always 1.
            TSDF_HOST_TIME(2);
            TSDF_TRY(B.prepare_batch(&bts[jp % kSets], depth, dk, color, TSDF_COLOR_RGB8, H, W,
                                     K, Tinv, nullptr, 1.0, flags, f0, n, jp % kSlots));
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
            sg.list_i = B.list_set[set_of(L)];
            sg.count_i = B.count_set[set_of(L)];
            sg.res_i = h->d_res + (size_t)set_of(L) * B.n_bricks;
        }
        if (has_c) {
            sg.list_c = B.list_set[set_of(L + 1)];
            sg.count_c = B.count_set[set_of(L + 1)];
            sg.res_c = h->d_res + (size_t)set_of(L + 1) * B.n_bricks;
        }
        if (has_p) sg.count_p = B.count_set[set_of(jp)];
        // the arrival counter of the commit (a word the prep of that set reset)
        sg.done = has_c ? sg.count_c + kDoneWordC : has_i ? sg.count_i + kDoneWord : nullptr;
        const long long grid = (long long)sg.gi + sg.gc + (has_p ? (long long)sg.ptx * sg.pty * bp.n : 0);
        if (grid >= (1ll << 31)) return set_error(TSDF_E_ARG, "fused grid too large");
        // the previous deferred batch's overflow check (its report; an exact re-run if it skipped
        // bricks) comes before this batch's integrate -- after this call's own ingest, prep and cull
        // were issued, so they overlap the previous batch on the GPU
        if (has_i && h->pend.on) TSDF_TRY(hash_settle(h));
        if (has_i || has_c) {
            // every launch with a cull allocates (its cull inserts the next batch's new blocks) and
            // every integrate may skip bricks: each such launch reports its pool state
            if (!sync && has_c) TSDF_TRY(async_room(h, h->seq));
            if (sync && !has_i) TSDF_TRY(ensure_room(h, true));  // (the call's first cull: last known state)
            sg.seq = h->seq++;
        } else {
            sg.seq = -1;
        }
        hipEvent_t e0 = nullptr;
        if (has_i) TSDF_TRY(B.prof.begin(B.stream, &e0));
        const FusedHashArgs args{B.vol, bi, bc, bp, B.pool, h->t, B.stats, sg};
        TSDF_HOST_TIME(3);
        // (u32 colour registers where the table's blocks are canonical, tsdf_device.h)
        const bool cu = TSDF_COLOR_U32 && B.vol.canon;
        if (tex) {
            if (cu) hipLaunchKernelGGL((k_fused_hash<2, true>), dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
            else hipLaunchKernelGGL(k_fused_hash<2>, dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
        } else if (dk == TSDF_DEPTH_U16_MM) {
            if (cu) hipLaunchKernelGGL((k_fused_hash<0, true>), dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
            else hipLaunchKernelGGL(k_fused_hash<0>, dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
        } else {
            if (cu) hipLaunchKernelGGL((k_fused_hash<1, true>), dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
            else hipLaunchKernelGGL(k_fused_hash<1>, dim3((unsigned)grid), dim3(kFusedHashWG), 0, B.stream, args);
        }
        TSDF_HIP(hipGetLastError());
        if (!has_i) continue;
        TSDF_TRY(B.prof.end(B.stream, e0));
        B.frames += bi.n;
        if (later) {
            TSDF_TRY(B.end_batch(flags, L % kSlots));
            h->pend.bt = bi;
            h->pend.dk = dk;
            h->pend.ck = TSDF_COLOR_RGB8;
            h->pend.seq = sg.seq;
            h->pend.on = true;
        } else if (sync) {
            TSDF_TRY(hash_after_batch(h, bi, dk, TSDF_COLOR_RGB8));
            TSDF_TRY(B.end_batch(flags, L % kSlots));
            TSDF_TRY(ensure_room(h, true));
        } else {
            TSDF_TRY(B.end_batch(flags, L % kSlots));
        }
    }
    // the blocks the call's culls inserted that no frame gave an entry (after the last launch, which
    // has no cull: no claim word is pending)
    TSDF_HOST_TIME(4);
    hipLaunchKernelGGL(k_free_unused, dim3(256), dim3(256), 0, B.stream, B.vol, h->t);
    TSDF_HIP(hipGetLastError());
    TSDF_HIP(hipMemsetAsync(&h->t.st->n_inserted, 0, sizeof(long long), B.stream));
    return TSDF_OK;
}

int hash_run(tsdf_hash* h, int n_frames, const void* depth, int dk, const void* color, int ck,
             int H, int W, const double* K, const double* Tinv, int flags) {
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    const unsigned cull_grid = h->t.owned ? (unsigned)std::max(1, (h->t.n_owned + 63) / 64) : B.cull_grid();
    const bool sync = !(flags & TSDF_ASYNC);
    if (!sync && h->rb_used < 0 && n_frames > B.batch && B.prestaged < 0) {
        // A fresh table's first asynchronous call: its first batch runs synchronously (the pool
        // grows exactly and skipped bricks re-run), so the growth of the batches in flight is
        // known before any launch depends on a lagging report.
        const int nbat = B.batch;
        TSDF_TRY(hash_run(h, nbat, depth, dk, color, ck, H, W, K, Tinv, flags & ~TSDF_ASYNC));
        depth = (const char*)depth + frame_bytes_depth(dk, H, W) * nbat;
        color = (const char*)color + frame_bytes_color(ck, H, W) * nbat;
        Tinv += 16 * nbat;
        n_frames -= nbat;
    }
    if (sync && h->async_pending) TSDF_TRY(take_overflow(h));  // before any replay of this call
    if (!sync) h->async_pending = true;
    TSDF_TRY(B.begin_call(depth, frame_bytes_depth(dk, H, W) * n_frames, color,
                          frame_bytes_color(ck, H, W) * n_frames, flags));
    CallGuard guard(B, flags);
    B.note_frames(ck, nullptr, n_frames, 1.0);
    // (the fused launch is built for power-of-two table sizes: every device table is one)
    const auto p2 = [](long long n) { return n > 0 && (n & (n - 1)) == 0; };
    bool fused = h->fused && ck == TSDF_COLOR_RGB8 && W % 4 == 0 && n_frames > 0 && p2(h->t.capacity) &&
                 p2(h->t.shard_cap);
    if (fused && (flags & TSDF_DEVICE_PTRS))
        fused = (uintptr_t)depth % (dk == TSDF_DEPTH_U16_MM ? 8 : 16) == 0 && (uintptr_t)color % 4 == 0 &&
                ((size_t)H * W) % 4 == 0;
    if (!fused && h->pend.on) TSDF_TRY(hash_settle(h));  // (the in-line path checks each batch at once)
    if (fused) {
        TSDF_TRY(hash_run_fused(h, n_frames, depth, dk, color, H, W, K, Tinv, flags));
        TSDF_TRY(guard.finish());
        if (sync && !h->pend.on) TSDF_HIP(hipStreamSynchronize(B.stream));
        return TSDF_OK;
    }
    B.use_set(0);
    const int nbat = B.batch;
    for (int f0 = 0; f0 < n_frames; f0 += nbat) {
        Batch bt;
        const int n = n_frames - f0 < nbat ? n_frames - f0 : nbat;
        const int slot = (f0 / nbat) % kSlots;
        // HashTable.integrate ignores obs_weight (hash_fusion.py:141,145): always 1.
        TSDF_TRY(B.prepare_batch(&bt, depth, dk, color, ck, H, W, K, Tinv, nullptr, 1.0, flags, f0, n, slot));
        TSDF_TRY(B.launch_prep(bt, dk, ck, W, H, B.stream));
        hipLaunchKernelGGL((k_cull<true>), dim3(cull_grid), dim3(kCullWG), 0, B.stream, B.vol, bt, h->t, B.list,
                           B.count, B.stats);
        TSDF_HIP(hipGetLastError());
        if (!sync) TSDF_TRY(async_room(h, h->seq));
        hipEvent_t e0;
        TSDF_TRY(B.prof.begin(B.stream, &e0));
        launch_integrate(h, bt, dk, ck, B.list, B.count, 0);
        TSDF_HIP(hipGetLastError());
        TSDF_TRY(B.prof.end(B.stream, e0));
        hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, B.stream, h->t.st, (long long)h->t.max_blocks,
                           h->t.rb, h->seq++, (const unsigned*)B.count);
        TSDF_HIP(hipGetLastError());
        B.frames += n;
        if (!sync) {
            TSDF_TRY(B.end_batch(flags, slot));
            continue;
        }
        TSDF_TRY(hash_after_batch(h, bt, dk, ck));
        TSDF_TRY(B.end_batch(flags, slot));  // the overflow re-runs above read this batch's frames
        TSDF_TRY(ensure_room(h, true));
    }
    TSDF_TRY(guard.finish());
    if (sync) TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

// The pending deferred batch's overflow check: grow the table / pool and re-run its skipped
// bricks exactly (hash_after_batch), then the load-factor policy.  Nothing has been launched on
// the handle since that batch, so its frames and prepped buffers are intact.
// The batch's integrate launch reported its pool state into page-locked host memory (PoolReport):
// without overflow the check is that report alone -- no stream synchronisation, no device read --
// and the load-factor policy on its counts; with overflow, the exact synchronous re-run.
int hash_settle(tsdf_hash* h) {
    if (!h->pend.on) return TSDF_OK;
    h->pend.on = false;
    PoolReport r;
    TSDF_TRY(wait_report(h, h->pend.seq, &r));
    if (r.n_overflow == 0) {
        h->host_st.pool_top = r.pool_top;
        h->host_st.free_count = r.free_count;
        h->host_st.n_overflow = 0;
        h->host_st.cursor = 0;
        h->tomb_est = table_tombs(h, h->pend.seq, r.tombs);
        h->host_st.tombs = h->tomb_est;
        return ensure_room(h, true);
    }
    TSDF_TRY(hash_after_batch(h, h->pend.bt, h->pend.dk, h->pend.ck));
    TSDF_TRY(ensure_room(h, true));
    return TSDF_OK;
}

// Run the deferred frames (TSDF_DEFER) as one batch from their bounce slot.  wait: synchronously
// (every entry point before it touches the state); otherwise (the per-frame integrate that filled
// the batch) the overflow check is left to the next call, so the host collects the next frames
// while the GPU integrates these -- either way a full table or pool is grown and the skipped
// bricks re-run exactly before any later frame is integrated.
int hash_flush(tsdf_hash* h, bool wait = true) {
    Base& B = h->b;
#ifdef TSDF_HOST_TIMES
    if (!wait && B.dfr.n) g_host_us[5] += 1.0;
    HostTimer whole(wait || !B.dfr.n ? 7 : 0);
#endif
    // (wait = false: a pending batch is settled inside hash_run, right before this batch's
    // integrate launch, once this batch's ingest / prep / cull are queued behind it)
    if (wait || B.dfr.n == 0) TSDF_TRY(hash_settle(h));
    if (B.dfr.n == 0) return TSDF_OK;
    const Base::Deferred d = B.dfr;
    B.dfr.n = 0;
    B.prestaged = d.slot;
    B.pre_copied = d.copied;
    const int r = hash_run(h, d.n, B.hst_depth[d.slot], d.dk, B.hst_color[d.slot], d.ck, d.H, d.W, d.K, d.T,
                           wait ? 0 : kCheckLater);
    B.prestaged = -1;
    B.pre_copied = 0;
    TSDF_TRY(r);
    if (wait) TSDF_TRY(hash_settle(h));
    return TSDF_OK;
}

int upload(tsdf_hash* h, const void* src, size_t bytes, void** dst) {
    *dst = nullptr;
    if (!src || !bytes) return TSDF_OK;
    TSDF_HIP(hipMalloc(dst, bytes));
    TSDF_HIP(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, h->b.stream));
    return TSDF_OK;
}

// Find-or-insert of distinct block keys (room first: the reference resizes before inserting,
// hash_fusion.py:208-209); *dblk / *dslot: device arrays (owned by bufs) of each key's block and
// slot.  Stream-ordered: the caller's kernels that use them follow on the handle's stream.
int insert_block_keys(tsdf_hash* h, const std::vector<unsigned long long>& keys, DevBufs& bufs, void** dblk,
                      void** dslot) {
    Base& B = h->b;
    const long long nk = (long long)keys.size();
    TSDF_TRY(read_state(h));
    InfoDev inf{};
    TSDF_TRY(info_raw(h, &inf));
    TSDF_TRY(table_room(h, (long long)inf.used, nk, (long long)inf.tomb));
    if (h->host_st.pool_top + nk > h->t.max_blocks - h->host_st.free_count)
        TSDF_TRY(grow_pool(h, pool_target(h, h->host_st.pool_top + 2 * nk)));
    void* dkeys;
    TSDF_TRY(upload(h, keys.data(), sizeof(unsigned long long) * nk, &dkeys));
    bufs.add(dkeys);
    TSDF_HIP(hipMalloc(dblk, sizeof(int) * (nk ? nk : 1)));
    bufs.add(*dblk);
    TSDF_HIP(hipMalloc(dslot, sizeof(long long) * (nk ? nk : 1)));
    bufs.add(*dslot);
    if (nk == 0) return TSDF_OK;
    hipLaunchKernelGGL(k_insert_blocks, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, B.stream, h->t,
                       B.pool, (const unsigned long long*)dkeys, (long long)nk, (int*)*dblk, (long long*)*dslot);
    TSDF_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, B.stream, h->t.st, (long long)h->t.max_blocks,
                       (PoolReport*)nullptr, -1ll, (const unsigned*)nullptr);
    TSDF_HIP(hipGetLastError());
    return TSDF_OK;
}

// unique packed block keys of the in-volume voxels of ijk
std::vector<unsigned long long> unique_blocks(const Vol& v, const int64_t* ijk, int64_t n) {
    std::vector<unsigned long long> keys;
    keys.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t x = ijk[3 * i], y = ijk[3 * i + 1], z = ijk[3 * i + 2];
        if (x < 0 || y < 0 || z < 0 || x >= v.dims[0] || y >= v.dims[1] || z >= v.dims[2]) continue;
        keys.push_back(pack_key((int)(x >> 3), (int)(y >> 3), (int)(z >> 3)));
    }
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    return keys;
}

}  // namespace

extern "C" {

int tsdf_hash_create(const int64_t dims[3], const float origin[3], double voxel_size, double trunc,
                     int64_t capacity, int64_t max_blocks, int int_bits, int shard, int n_shards,
                     int device, tsdf_hash_t** out) {
    if (!dims || !origin || !out) return set_error(TSDF_E_ARG, "null pointer");
    *out = nullptr;
    if (capacity <= 0 || capacity > (1ll << 40)) return set_error(TSDF_E_ARG, "capacity out of range");
    if (int_bits != 32 && int_bits != 64) return set_error(TSDF_E_ARG, "int_bits must be 32 or 64");
    if (n_shards < 1 || shard < 0 || shard >= n_shards) return set_error(TSDF_E_ARG, "bad shard %d/%d", shard, n_shards);
    tsdf_hash* h = new tsdf_hash();
    int r = h->b.init(device, dims, nullptr, origin, voxel_size, trunc);
    Table& t = h->t;
    if (r == TSDF_OK) {
        h->b.vol.shard = shard;
        h->b.vol.n_shards = n_shards;
        r = h->b.set_batch(n_shards > 1 ? kMaxBatch : kFullBatch);
        if (max_blocks <= 0) max_blocks = std::min<long long>(h->b.n_bricks, 1 << 16);
        max_blocks = std::max<long long>(std::min<long long>(max_blocks, h->b.n_bricks), 64);
        h->map_size = capacity;
        t.capacity = next_pow2(capacity);
        t.shard_cap = t.capacity;
        t.max_blocks = max_blocks;
        t.int_bits = int_bits;
        t.overflow_cap = (int)std::min<long long>(h->b.n_bricks, 1ll << 30);
        hipError_t e = hipMalloc(&t.keys, sizeof(unsigned long long) * t.capacity);
        if (e == hipSuccess) e = hipMalloc(&t.vals, sizeof(int) * t.capacity);
        if (e == hipSuccess) e = hipMalloc(&t.overflow, sizeof(ListEntry) * (size_t)t.overflow_cap);
        if (e == hipSuccess) e = hipMalloc(&t.st, sizeof(PoolState));
        if (e == hipSuccess && n_shards > 1) {
            // the bricks this bucket-range shard owns (fixed at create, Table::shard_cap), for the
            // cull (cull_owned): increasing brick index
            const Vol& v = h->b.vol;
            std::vector<int> own;
            own.reserve((size_t)(h->b.n_bricks / n_shards + 64));
            for (int bx = 0; bx < v.nb[0]; ++bx)
                for (int by = 0; by < v.nb[1]; ++by)
                    for (int bz = 0; bz < v.nb[2]; ++bz)
                        if (shard_of(ref_hash(bx, by, bz, t.shard_cap, int_bits), n_shards, t.shard_cap) == shard)
                            own.push_back((bx * v.nb[1] + by) * v.nb[2] + bz);
            t.n_owned = (int)own.size();
            e = hipMalloc((void**)&t.owned, sizeof(int) * std::max<size_t>(own.size(), 1));
            if (e == hipSuccess && !own.empty())
                e = hipMemcpy((void*)t.owned, own.data(), sizeof(int) * own.size(), hipMemcpyHostToDevice);
        }
        // the pool: address ranges for every brick of the volume, backed as it grows
        // (TSDF_HASH_VMM=0: plain allocations, grown by copy)
        const char* ev = getenv("TSDF_HASH_VMM");
        const size_t nb = (size_t)h->b.n_bricks;
        h->vmm = e == hipSuccess && !(ev && atoi(ev) == 0) &&
                 h->va[0].reserve(device, nb * kBrickVox * sizeof(float)) &&
                 h->va[1].reserve(device, nb * kBrickVox * sizeof(float)) &&
                 h->va[2].reserve(device, nb * kBrickVox * sizeof(float)) &&
                 h->va[3].reserve(device, nb * 8 * sizeof(unsigned long long)) &&
                 h->va[4].reserve(device, nb * sizeof(int));
        if (h->vmm && h->map_pool(max_blocks) != TSDF_OK) {  // fall back to plain allocations
            for (auto& v : h->va) v.release();
            h->vmm = false;
        }
        if (!h->vmm)
            for (auto& v : h->va) v.release();
        if (h->vmm) {
            h->b.pool.tsdf = (float*)h->va[0].base;
            h->b.pool.weight = (float*)h->va[1].base;
            h->b.pool.color = (float*)h->va[2].base;
            t.occ = (unsigned long long*)h->va[3].base;
            t.free_list = (int*)h->va[4].base;
        } else {
            if (e == hipSuccess) e = hipMalloc(&t.occ, sizeof(unsigned long long) * 8 * max_blocks);
            if (e == hipSuccess) e = hipMalloc(&t.free_list, sizeof(int) * max_blocks);
            if (e == hipSuccess) e = hipMalloc(&h->b.pool.tsdf, sizeof(float) * kBrickVox * max_blocks);
            if (e == hipSuccess) e = hipMalloc(&h->b.pool.weight, sizeof(float) * kBrickVox * max_blocks);
            if (e == hipSuccess) e = hipMalloc(&h->b.pool.color, sizeof(float) * kBrickVox * max_blocks);
        }
        if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_rb, sizeof(PoolReport) * kReports, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            std::memset(h->h_rb, 0, sizeof(PoolReport) * kReports);
            e = hipHostGetDevicePointer((void**)&t.rb, h->h_rb, 0);
        }
        if (e != hipSuccess)
            r = set_error(e == hipErrorOutOfMemory ? TSDF_E_OOM : TSDF_E_HIP, "hash allocation: %s",
                          hipGetErrorString(e));
    }
    if (const char* e = getenv("TSDF_PIPELINE")) h->fused = atoi(e) != 0;  // 0: in-line kernels
    if (const char* e = getenv("TSDF_HASH_VMM_FAIL")) h->vmm_fail_at = atoi(e);  // (after the initial mapping)
    if (const char* e = getenv("TSDF_HASH_ASYNC_GROW")) h->async_grow = atoi(e) != 0;
    if (const char* e = getenv("TSDF_HASH_MAX_LOAD")) {
        const double ml = atof(e);
        if (ml > 0.0 && ml < 1.0) h->max_load = ml;
    }
    if (r == TSDF_OK) r = tsdf_hash_reset(h);
    if (r != TSDF_OK) {
        std::string keep = tsdf_last_error();
        tsdf_hash_destroy(h);
        set_error(r, "%s", keep.c_str());
        return r;
    }
    *out = h;
    return TSDF_OK;
}

int tsdf_hash_destroy(tsdf_hash_t* h) {
    if (!h) return TSDF_OK;
    (void)hipSetDevice(h->b.device);
    h->b.release();
    void* ps[] = {h->t.keys, h->t.vals, h->t.overflow, h->t.st, h->d_list, h->d_res, h->d_ins, (void*)h->t.owned};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    if (h->vmm) {
        for (auto& v : h->va) v.release();
    } else {
        void* pool[] = {h->t.occ, h->t.free_list, h->b.pool.tsdf, h->b.pool.weight, h->b.pool.color};
        for (void* p : pool)
            if (p) (void)hipFree(p);
    }
    for (const auto& r : h->retired_va) (void)hipMemAddressFree(r.first, r.second);
    if (h->h_rb) (void)hipHostFree(h->h_rb);
    delete h;
    return TSDF_OK;
}

int tsdf_hash_reset(tsdf_hash_t* h) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    Base& B = h->b;
    B.dfr.n = 0;  // deferred frames are dropped with the state
    h->pend.on = false;
    TSDF_HIP(hipSetDevice(B.device));
    hipLaunchKernelGGL(k_fill_keys, dim3(2048), dim3(256), 0, B.stream, h->t.keys, h->t.vals,
                       (long long)h->t.capacity);
    TSDF_HIP(hipGetLastError());
    TSDF_HIP(hipMemsetAsync(h->t.st, 0, sizeof(PoolState), B.stream));
    TSDF_HIP(hipMemsetAsync(B.stats, 0, sizeof(unsigned long long) * kNStat * kStatSpread, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    B.frames = 0;
    std::memset(&h->host_st, 0, sizeof(h->host_st));
    h->rb_used = -1;
    std::fill(std::begin(h->deltas), std::end(h->deltas), 0ll);
    h->n_delta = 0;
    h->tomb_est = 0;
    h->async_pending = false;
    B.vol.canon = 1;
    return TSDF_OK;
}

int tsdf_hash_integrate(tsdf_hash_t* h, const void* depth, int depth_kind, const void* color,
                        int color_kind, int height, int width, const double K[9],
                        const double world_to_cam[16], int flags) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_TRY(check_frame_args(depth, depth_kind, color, color_kind, height, width, K, world_to_cam));
    TSDF_HIP(hipSetDevice(h->b.device));
    Base& B = h->b;
    if (flags & TSDF_DEFER) {
        if (flags & TSDF_DEVICE_PTRS) return set_error(TSDF_E_ARG, "TSDF_DEFER takes host frames only");
        if (B.dfr.n > 0 && !B.defer_same(depth_kind, color_kind, height, width, K)) TSDF_TRY(hash_flush(h));
        // a pending batch's re-run reads its staging slots: settle it before they are reallocated
        if (h->pend.on && !B.stage_fits(depth_kind, color_kind, height, width)) TSDF_TRY(hash_settle(h));
        // HashTable.integrate ignores obs_weight (hash_fusion.py:141,145): always 1
        int r = B.defer_push(depth, depth_kind, color, color_kind, height, width, K, world_to_cam, 1.0);
        if (r == Base::kDeferFlush) {  // the batch's frames went as u16 and this one cannot
            TSDF_TRY(hash_flush(h));
            r = B.defer_push(depth, depth_kind, color, color_kind, height, width, K, world_to_cam, 1.0);
        }
        TSDF_TRY(r);
        if (B.dfr.n == B.defer_frames) TSDF_TRY(hash_flush(h, false));
        return TSDF_OK;
    }
    TSDF_TRY(hash_flush(h));
    return hash_run(h, 1, depth, depth_kind, color, color_kind, height, width, K, world_to_cam, flags);
}

int tsdf_hash_integrate_batch(tsdf_hash_t* h, int n_frames, const void* depth, int depth_kind,
                              const void* color, int color_kind, int height, int width,
                              const double K[9], const double* world_to_cam, int flags) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    if (n_frames < 0) return set_error(TSDF_E_ARG, "n_frames < 0");
    if (n_frames == 0) return TSDF_OK;
    TSDF_TRY(check_frame_args(depth, depth_kind, color, color_kind, height, width, K, world_to_cam));
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    return hash_run(h, n_frames, depth, depth_kind, color, color_kind, height, width, K,
                    world_to_cam, flags);
}

int tsdf_hash_lookup(tsdf_hash_t* h, const int64_t* ijk, int64_t n, float* tsdf_, float* weight_,
                     float* color_, uint8_t* found) {
    if (!h || (n > 0 && (!ijk || !found)) || n < 0) return set_error(TSDF_E_ARG, "bad arguments");
    if (n == 0) return TSDF_OK;
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    DevBufs bufs;
    void *dijk, *dt = nullptr, *dw = nullptr, *dc = nullptr, *df = nullptr;
    TSDF_TRY(upload(h, ijk, sizeof(int64_t) * 3 * n, &dijk));
    bufs.add(dijk);
    if (tsdf_) { TSDF_HIP(hipMalloc(&dt, sizeof(float) * n)); bufs.add(dt); }
    if (weight_) { TSDF_HIP(hipMalloc(&dw, sizeof(float) * n)); bufs.add(dw); }
    if (color_) { TSDF_HIP(hipMalloc(&dc, sizeof(float) * n)); bufs.add(dc); }
    TSDF_HIP(hipMalloc(&df, n));
    bufs.add(df);
    hipLaunchKernelGGL(k_lookup, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, B.stream, B.vol, h->t,
                       B.pool, (const long long*)dijk, (long long)n, (float*)dt, (float*)dw, (float*)dc,
                       (unsigned char*)df);
    TSDF_HIP(hipGetLastError());
    if (tsdf_) TSDF_HIP(hipMemcpyAsync(tsdf_, dt, sizeof(float) * n, hipMemcpyDeviceToHost, B.stream));
    if (weight_) TSDF_HIP(hipMemcpyAsync(weight_, dw, sizeof(float) * n, hipMemcpyDeviceToHost, B.stream));
    if (color_) TSDF_HIP(hipMemcpyAsync(color_, dc, sizeof(float) * n, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipMemcpyAsync(found, df, n, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

int tsdf_hash_insert(tsdf_hash_t* h, const int64_t* ijk, int64_t n, const float* tsdf_,
                     const float* weight_, const float* color_, int64_t* slot, int32_t* local) {
    if (!h || n < 0 || (n > 0 && !ijk)) return set_error(TSDF_E_ARG, "bad arguments");
    if (n == 0) return TSDF_OK;
    Base& B = h->b;
    const Vol& v = B.vol;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t x = ijk[3 * i], y = ijk[3 * i + 1], z = ijk[3 * i + 2];
        if (x < 0 || y < 0 || z < 0 || x >= v.dims[0] || y >= v.dims[1] || z >= v.dims[2])
            return set_error(TSDF_E_ARG, "voxel (%lld,%lld,%lld) outside the volume %dx%dx%d",
                             (long long)x, (long long)y, (long long)z, v.dims[0], v.dims[1], v.dims[2]);
    }
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    std::vector<unsigned long long> keys = unique_blocks(v, ijk, n);
    const long long nk = (long long)keys.size();
    DevBufs bufs;
    void *dblk = nullptr, *dslot = nullptr, *dijk, *dt, *dw, *dc;
    TSDF_TRY(insert_block_keys(h, keys, bufs, &dblk, &dslot));
    TSDF_TRY(upload(h, ijk, sizeof(int64_t) * 3 * n, &dijk));
    bufs.add(dijk);
    TSDF_TRY(upload(h, tsdf_, tsdf_ ? sizeof(float) * n : 0, &dt));
    bufs.add(dt);
    TSDF_TRY(upload(h, weight_, weight_ ? sizeof(float) * n : 0, &dw));
    bufs.add(dw);
    TSDF_TRY(upload(h, color_, color_ ? sizeof(float) * n : 0, &dc));
    bufs.add(dc);
    hipLaunchKernelGGL(k_set_voxels, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, B.stream, B.vol, h->t,
                       B.pool, (const long long*)dijk, (long long)n, (const float*)dt, (const float*)dw,
                       (const float*)dc);
    TSDF_HIP(hipGetLastError());
    std::vector<int> blk(nk);
    std::vector<long long> sl(nk);
    TSDF_HIP(hipMemcpyAsync(blk.data(), dblk, sizeof(int) * nk, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipMemcpyAsync(sl.data(), dslot, sizeof(long long) * nk, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    for (long long i = 0; i < nk; ++i)
        if (blk[i] < 0) return set_error(TSDF_E_CAPACITY, "hash insert failed (table or pool full)");
    if (weight_ || color_) TSDF_TRY(recheck_canon(h));
    if (slot || local) {
        for (int64_t i = 0; i < n; ++i) {
            const int64_t x = ijk[3 * i], y = ijk[3 * i + 1], z = ijk[3 * i + 2];
            const unsigned long long k = pack_key((int)(x >> 3), (int)(y >> 3), (int)(z >> 3));
            const long long j = std::lower_bound(keys.begin(), keys.end(), k) - keys.begin();
            if (slot) slot[i] = sl[j];
            if (local) local[i] = (int32_t)(((x & 7) * 8 + (y & 7)) * 8 + (z & 7));
        }
    }
    return TSDF_OK;
}

int tsdf_hash_remove(tsdf_hash_t* h, const int64_t* ijk, int64_t n, uint8_t* removed) {
    if (!h || n < 0 || (n > 0 && !ijk)) return set_error(TSDF_E_ARG, "bad arguments");
    if (n == 0) return TSDF_OK;
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    std::vector<unsigned long long> keys = unique_blocks(B.vol, ijk, n);
    DevBufs bufs;
    void *dijk, *dkeys, *drem = nullptr;
    TSDF_TRY(upload(h, ijk, sizeof(int64_t) * 3 * n, &dijk));
    bufs.add(dijk);
    if (removed) {
        TSDF_HIP(hipMalloc(&drem, n));
        bufs.add(drem);
    }
    hipLaunchKernelGGL(k_remove_voxels, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, B.stream, B.vol,
                       h->t, (const long long*)dijk, (long long)n, (unsigned char*)drem);
    TSDF_HIP(hipGetLastError());
    if (!keys.empty()) {
        TSDF_TRY(upload(h, keys.data(), sizeof(unsigned long long) * keys.size(), &dkeys));
        bufs.add(dkeys);
        hipLaunchKernelGGL(k_free_empty, dim3((unsigned)((keys.size() + 255) / 256)), dim3(256), 0, B.stream,
                           h->t, (const unsigned long long*)dkeys, (long long)keys.size());
        TSDF_HIP(hipGetLastError());
    }
    if (removed) TSDF_HIP(hipMemcpyAsync(removed, drem, n, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

int tsdf_hash_resize(tsdf_hash_t* h, int64_t new_capacity) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    InfoDev inf{};
    TSDF_TRY(info_raw(h, &inf));
    if (new_capacity <= (int64_t)inf.used) return set_error(TSDF_E_ARG, "new capacity too small");
    if (new_capacity > (1ll << 40)) return set_error(TSDF_E_ARG, "capacity out of range");
    const long long slots = next_pow2(new_capacity);
    if (slots != h->t.capacity) TSDF_TRY(resize_table(h, slots));
    h->map_size = new_capacity;
    return TSDF_OK;
}

int tsdf_hash_info(tsdf_hash_t* h, tsdf_hash_info_t* out) {
    if (!h || !out) return set_error(TSDF_E_ARG, "null pointer");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    InfoDev inf{};
    TSDF_TRY(info_raw(h, &inf));
    TSDF_TRY(read_state(h));
    out->capacity = h->map_size;
    out->slots = h->t.capacity;
    out->pool_mapped = h->vmm ? 1 : 0;
    out->used = (int64_t)inf.used;
    out->tombstones = (int64_t)inf.tomb;
    out->displaced = (int64_t)inf.displaced;
    out->max_probe = (int64_t)inf.max_probe;
    out->blocks_in_pool = h->host_st.pool_top;
    out->pool_capacity = h->t.max_blocks;
    out->entries = (int64_t)inf.entries;
    return TSDF_OK;
}

int tsdf_hash_get_dense(tsdf_hash_t* h, float* tsdf_, float* weight_, float* color_) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    const size_t n = (size_t)B.vol.dims[0] * B.vol.dims[1] * B.vol.dims[2];
    DevBufs bufs;
    void *dt = nullptr, *dw = nullptr, *dc = nullptr;
    if (tsdf_) { TSDF_HIP(hipMalloc(&dt, n * sizeof(float))); bufs.add(dt); }
    if (weight_) { TSDF_HIP(hipMalloc(&dw, n * sizeof(float))); bufs.add(dw); }
    if (color_) { TSDF_HIP(hipMalloc(&dc, n * sizeof(float))); bufs.add(dc); }
    hipLaunchKernelGGL(k_fill_dense, dim3(4096), dim3(256), 0, B.stream, (float*)dt, (float*)dw, (float*)dc, n);
    TSDF_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_to_dense, dim3(4096), dim3(256), 0, B.stream, B.vol, h->t, B.pool, (float*)dt,
                       (float*)dw, (float*)dc);
    TSDF_HIP(hipGetLastError());
    if (tsdf_) TSDF_HIP(hipMemcpyAsync(tsdf_, dt, n * sizeof(float), hipMemcpyDeviceToHost, B.stream));
    if (weight_) TSDF_HIP(hipMemcpyAsync(weight_, dw, n * sizeof(float), hipMemcpyDeviceToHost, B.stream));
    if (color_) TSDF_HIP(hipMemcpyAsync(color_, dc, n * sizeof(float), hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    return TSDF_OK;
}

int tsdf_hash_to_dense(tsdf_hash_t* h, tsdf_dense_t* d) {
    if (!h || !d) return set_error(TSDF_E_ARG, "null handle");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    TSDF_TRY(tsdf_dense_sync(d));  // (runs the dense handle's deferred frames first)
    Base& D = *dense_base(d);
    // the same lattice: dims, contiguous columns, origin, voxel size and truncation (a handle with
    // other bounds but equal dims would be filled with a misplaced volume)
    bool same = D.vol.xstride == kBrickEdge && D.vol.xodd == kBrickEdge && D.vol.vs == B.vol.vs &&
                D.vol.trunc == B.vol.trunc;
    for (int a = 0; a < 3; ++a)
        same = same && D.vol.dims[a] == B.vol.dims[a] && D.vol.off[a] == 0 && B.vol.off[a] == 0 &&
               D.vol.origin[a] == B.vol.origin[a];
    if (!same)
        return set_error(TSDF_E_ARG, "the dense handle must be an unsharded volume of the hash's geometry "
                                     "(dims, origin, voxel size, truncation)");
    if (D.device != B.device) return set_error(TSDF_E_ARG, "the handles live on different devices");
    TSDF_TRY(tsdf_dense_reset(d));  // (1, 0, 0) everywhere, then the live blocks' entries
    hipLaunchKernelGGL(k_to_bricks, dim3(4096), dim3(256), 0, B.stream, B.vol, h->t, B.pool, D.pool);
    TSDF_HIP(hipGetLastError());
    TSDF_HIP(hipStreamSynchronize(B.stream));
    D.vol.canon = B.vol.canon;
    return TSDF_OK;
}

int tsdf_hash_sync(tsdf_hash_t* h) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    TSDF_HIP(hipStreamSynchronize(h->b.stream));
    if (h->async_pending) TSDF_TRY(take_overflow(h));
    return TSDF_OK;
}

int tsdf_hash_trim(tsdf_hash_t* h) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_TRY(tsdf_hash_sync(h));
    return trim_pool(h);
}

int tsdf_hash_stats(tsdf_hash_t* h, tsdf_stats_t* out, int reset) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    return h->b.read_stats(out, reset);
}

int tsdf_hash_frames_per_launch(tsdf_hash_t* h, int* n) {
    if (!h || !n) return set_error(TSDF_E_ARG, "null pointer");
    *n = h->b.batch;
    return TSDF_OK;
}

int tsdf_hash_set_profiling(tsdf_hash_t* h, int on) {
    if (!h) return set_error(TSDF_E_ARG, "null handle");
    TSDF_HIP(hipSetDevice(h->b.device));
    TSDF_TRY(hash_flush(h));
    return h->b.set_profiling(on);
}

// Sparse export / import of whole blocks (the multi-GPU merge of bucket-range shards, DESIGN.md
// §6): only live blocks move, never the dense extent.
int tsdf_hash_export_blocks(tsdf_hash_t* h, int32_t* bxyz, float* tsdf_, float* weight_, float* color_,
                            uint64_t* occ, int64_t* n_blocks, int flags) {
    if (!h || !n_blocks) return set_error(TSDF_E_ARG, "null pointer");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    InfoDev inf{};
    TSDF_TRY(info_raw(h, &inf));
    const long long live = (long long)inf.used;
    if (!bxyz) {  // count only
        *n_blocks = live;
        return TSDF_OK;
    }
    if (*n_blocks < live) return set_error(TSDF_E_ARG, "output holds %lld blocks, %lld live", (long long)*n_blocks, live);
    const bool dev = (flags & TSDF_DEVICE_PTRS) != 0;
    DevBufs bufs;
    void* d[5] = {bxyz, tsdf_, weight_, color_, occ};
    const size_t sz[5] = {sizeof(int32_t) * 3, sizeof(float) * kBrickVox, sizeof(float) * kBrickVox,
                          sizeof(float) * kBrickVox, sizeof(uint64_t) * 8};
    if (!dev)
        for (int k = 0; k < 5; ++k)
            if (d[k]) {
                TSDF_HIP(hipMalloc(&d[k], sz[k] * (live ? live : 1)));
                bufs.add(d[k]);
            }
    unsigned long long* counter;
    TSDF_HIP(hipMalloc(&counter, sizeof(unsigned long long)));
    bufs.add(counter);
    TSDF_HIP(hipMemsetAsync(counter, 0, sizeof(unsigned long long), B.stream));
    hipLaunchKernelGGL(k_export_blocks, dim3(2048), dim3(256), 0, B.stream, h->t, B.pool, counter, live, (int*)d[0],
                       (float*)d[1], (float*)d[2], (float*)d[3], (unsigned long long*)d[4]);
    TSDF_HIP(hipGetLastError());
    unsigned long long got = 0;
    TSDF_HIP(hipMemcpyAsync(&got, counter, sizeof(got), hipMemcpyDeviceToHost, B.stream));
    if (!dev) {
        void* out[5] = {bxyz, tsdf_, weight_, color_, occ};
        for (int k = 0; k < 5; ++k)
            if (out[k]) TSDF_HIP(hipMemcpyAsync(out[k], d[k], sz[k] * live, hipMemcpyDeviceToHost, B.stream));
    }
    TSDF_HIP(hipStreamSynchronize(B.stream));
    if ((long long)got != live) return set_error(TSDF_E_HIP, "exported %llu blocks, expected %lld", got, live);
    *n_blocks = live;
    return TSDF_OK;
}

int tsdf_hash_import_blocks(tsdf_hash_t* h, const int32_t* bxyz, int64_t n_blocks, const float* tsdf_,
                            const float* weight_, const float* color_, const uint64_t* occ, int flags) {
    if (!h || n_blocks < 0 || (n_blocks > 0 && !bxyz)) return set_error(TSDF_E_ARG, "bad arguments");
    Base& B = h->b;
    TSDF_HIP(hipSetDevice(B.device));
    TSDF_TRY(hash_flush(h));
    if (n_blocks == 0) return TSDF_OK;
    const bool dev = (flags & TSDF_DEVICE_PTRS) != 0;
    std::vector<int32_t> hb((size_t)n_blocks * 3);
    if (dev) {
        TSDF_HIP(hipDeviceSynchronize());  // the caller's producer may be on another stream
        TSDF_HIP(hipMemcpy(hb.data(), bxyz, hb.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    } else {
        std::memcpy(hb.data(), bxyz, hb.size() * sizeof(int32_t));
    }
    std::vector<unsigned long long> keys((size_t)n_blocks);
    for (int64_t i = 0; i < n_blocks; ++i) {
        const int bx = hb[3 * i], by = hb[3 * i + 1], bz = hb[3 * i + 2];
        if (bx < 0 || by < 0 || bz < 0 || bx >= B.vol.nb[0] || by >= B.vol.nb[1] || bz >= B.vol.nb[2])
            return set_error(TSDF_E_ARG, "block (%d,%d,%d) outside the volume", bx, by, bz);
        keys[i] = pack_key(bx, by, bz);
    }
    {
        std::vector<unsigned long long> u(keys);
        std::sort(u.begin(), u.end());
        if (std::adjacent_find(u.begin(), u.end()) != u.end()) return set_error(TSDF_E_ARG, "duplicate block in import");
    }
    DevBufs bufs;
    void *dblk = nullptr, *dslot = nullptr;
    TSDF_TRY(insert_block_keys(h, keys, bufs, &dblk, &dslot));
    const void* in[4] = {tsdf_, weight_, color_, occ};
    const size_t sz[4] = {sizeof(float) * kBrickVox, sizeof(float) * kBrickVox, sizeof(float) * kBrickVox,
                          sizeof(uint64_t) * 8};
    void* d[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int k = 0; k < 4; ++k) {
        if (!in[k]) continue;
        if (dev) {
            d[k] = (void*)in[k];
        } else {
            TSDF_TRY(upload(h, in[k], sz[k] * n_blocks, &d[k]));
            bufs.add(d[k]);
        }
    }
    hipLaunchKernelGGL(k_write_blocks, dim3(2048), dim3(256), 0, B.stream, h->t, B.pool, (const int*)dblk,
                       (long long)n_blocks, (const float*)d[0], (const float*)d[1], (const float*)d[2],
                       (const unsigned long long*)d[3]);
    TSDF_HIP(hipGetLastError());
    std::vector<int> blk((size_t)n_blocks);
    TSDF_HIP(hipMemcpyAsync(blk.data(), dblk, sizeof(int) * n_blocks, hipMemcpyDeviceToHost, B.stream));
    TSDF_HIP(hipStreamSynchronize(B.stream));
    for (int64_t i = 0; i < n_blocks; ++i)
        if (blk[i] < 0) return set_error(TSDF_E_CAPACITY, "hash import failed (table or pool full)");
    if (weight_ || color_) TSDF_TRY(recheck_canon(h));
    return TSDF_OK;
}

}  // extern "C"

#ifdef TSDF_WG_TIMES
// (diagnostic builds) the last fused hash launch's per-workgroup start / end / role|items
extern "C" int tsdf_diag_wg_times_hash(unsigned long long* out) {
    TSDF_HIP(hipDeviceSynchronize());
    TSDF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_times), sizeof(unsigned long long) * 4 * kWgTimes));
    static const std::vector<unsigned long long> zero(4 * (size_t)kWgTimes, 0ull);  // (read and cleared)
    TSDF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wg_times), zero.data(), sizeof(unsigned long long) * 4 * kWgTimes));
    return TSDF_OK;
}
#endif

#ifdef TSDF_HOST_TIMES
// (diagnostic builds) the drop-in flush's host times (g_host_us above), read and cleared
extern "C" int tsdf_diag_host_times(double* out) {
    for (int i = 0; i < 8; ++i) {
        out[i] = g_host_us[i];
        g_host_us[i] = 0.0;
    }
    return TSDF_OK;
}
#endif
