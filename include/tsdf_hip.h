/*
 * tsdf_hip.h -- C-ABI of the MI355X (gfx950) TSDF fusion hot path.
 *
 * The drop-in boundary for DiWu9/Union-Thesis-SLAM's integrate path: the reference binds its
 * device code from Python (PyCUDA SourceModule, grid_fusion.py:69-144, launched at :234-259);
 * this library is bound the same way, from Python, through ctypes
 * (union-thesis-slam_amd/tsdf_amd/_ffi.py).  Plain C types only: pointers, sizes, doubles.
 *
 * Conventions
 *   - Every function returns int: 0 = ok, negative = TSDF_E_* code; tsdf_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - A handle owns all of its device memory and one HIP stream on its device.  Host pointers
 *     are borrowed for the duration of the call only and must be C-contiguous.
 *   - Calls are synchronous (stream-synchronised before return) unless TSDF_ASYNC is passed;
 *     then the caller synchronises with tsdf_*_sync().  One handle per host thread.
 *   - Pointer residence is given per call by TSDF_DEVICE_PTRS: without it depth/colour are host
 *     pointers (copied H2D by the call); with it they are device pointers already in HBM.
 *   - Volumes are indexed like the reference: voxel (x, y, z), C-order (X, Y, Z), z fastest
 *     (grid_fusion.py:52-55,158-168).  The state lives in HBM as 8x8x8 bricks;
 *     the get/extract calls return C-order arrays.
 */
#ifndef TSDF_HIP_H
#define TSDF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------------------------ */
#define TSDF_OK 0
#define TSDF_E_ARG -1       /* invalid argument (shape, kind, null pointer) */
#define TSDF_E_HIP -2       /* a HIP runtime call failed (message has the HIP error string) */
#define TSDF_E_NODEV -3     /* no usable gfx950 device */
#define TSDF_E_CAPACITY -4  /* hash table / block pool full and could not grow */
#define TSDF_E_OOM -5       /* device allocation failed */

/* ---- input kinds and flags ---------------------------------------------------------------- */
#define TSDF_DEPTH_U16_MM 0 /* uint16 millimetres: metres = (double)mm / 1000.0 (grid_demo1.py:81-82) */
#define TSDF_DEPTH_F64_M 1  /* float64 metres, as handed to integrate() (grid_fusion.py:214) */
#define TSDF_COLOR_RGB8 0   /* uint8 (H,W,3) RGB; folded B*65536+G*256+R (grid_fusion.py:228-232) */
#define TSDF_COLOR_F32 1    /* float32 (H,W) already folded by the caller */

#define TSDF_DEVICE_PTRS 1  /* depth/colour pointers are device pointers */
#define TSDF_ASYNC 2        /* do not synchronise the handle's stream before returning */
#define TSDF_DEPTH_INVALID_65535 4 /* u16 depth: 65535 mm is invalid (0), the 7-Scenes convention
                                      of the demos (grid_demo1.py:82: depth_im[depth_im == 65.535] = 0) */
#define TSDF_DEFER 8        /* tsdf_*_integrate (host frames only): copy the frame into a pinned
                               staging batch and return; the batch runs (asynchronously, as one
                               temporally batched launch) once it holds 8 frames
                               (TSDF_DEFER_FRAMES overrides; a quarter of a 32-frame
                               launch, the host's copy grain) or at the next other call
                               on the handle -- the reference's one-integrate()-per-
                               frame loop (grid_demo1.py:76-87) at batched speed, same results.
                               f64-metre depth whose every value is exactly RN(k / 1000),
                               k < 65536 integer (png / 1000.), is staged as u16 millimetres.
                               Hash: a full table / pool found after a deferred batch is grown
                               and its skipped bricks re-run at the next call, before anything
                               else runs (exact, as for synchronous calls) */

typedef struct tsdf_dense tsdf_dense_t;
typedef struct tsdf_hash tsdf_hash_t;

/* Cumulative counters since create/reset (or the last tsdf_*_stats call with reset != 0). */
typedef struct {
    int64_t frames;           /* frames integrated */
    int64_t voxel_updates;    /* sum over frames of V_f (voxels whose tsdf/weight/colour changed) */
    int64_t bricks_visited;   /* bricks that passed the conservative frustum/depth cull */
    int64_t bricks_touched;   /* bricks with >= 1 updated voxel, summed over launches; the fused
                                 launches count each z-half wave that updated a voxel (up to two
                                 per brick) -- per-block counts: lookups */
    int64_t blocks_allocated; /* hash: blocks newly allocated */
    int64_t probe_steps;      /* hash: total linear-probe distance of block lookups */
    int64_t probe_max;        /* hash: longest probe distance seen */
    int64_t lookups;          /* hash: block lookups performed (fused launches: one per kept
                                 block per launch, by the cull's find-or-insert) */
    double kernel_ms;         /* integrate-kernel time from HIP events (profiling on only) */
    int64_t kernel_launches;  /* integrate-kernel launches timed */
    int64_t bricks_skipped;   /* hash: bricks a launch skipped for lack of table/pool space --
                                 re-run exactly after growing by a synchronous call (and counted
                                 here), reported as TSDF_E_CAPACITY by an asynchronous one; see
                                 tsdf_hash_integrate_batch */
    int64_t list_errors;      /* brick-list entries out of range, dropped by the integrate kernel
                                 (always 0 unless device memory was corrupted) */
    int64_t batch_voxels;     /* sum over launches of U_batch: the voxels updated at least once by
                                 the launch's temporal batch (<= voxel_updates; each such voxel's
                                 state is read and written once per launch -- the roofline's bytes) */
} tsdf_stats_t;

typedef struct {
    int64_t capacity;         /* the table size of the API (map_size: hash_function's modulus, doubled
                                 by double_table_size and the 0.75 load-factor policy) */
    int64_t used;             /* live block keys */
    int64_t tombstones;       /* removed keys not yet reclaimed by a rehash */
    int64_t displaced;        /* live keys not in their home slot ("collisions") */
    int64_t max_probe;        /* longest home-to-slot distance of a live key */
    int64_t blocks_in_pool;   /* blocks handed out by the pool (live + free list) */
    int64_t pool_capacity;    /* blocks the pool can hold before it must grow */
    int64_t entries;          /* voxel entries (occupancy bits set), = count_num_hash_entries */
    int64_t slots;            /* slots of the open-addressed device table: the power of two >= capacity */
    int64_t pool_mapped;      /* 1: the pool lives on reserved address ranges grown by mapping (VMM);
                                 0: plain allocations grown by copy */
} tsdf_hash_info_t;

const char* tsdf_last_error(void);
/* Build id of the loaded library: the first 16 hex digits of the sha256 of the sources it was
 * compiled from (csrc/, this header, the Makefile).  Profiles under profiles/ record the id of
 * the library they measured; bench.py quotes a profile's counters only for the same id. */
const char* tsdf_build_id(void);
int tsdf_device_count(int* n);

/* ---- dense grid: replaces TSDFVolume (grid_fusion.py:19-320) ------------------------------
 * dims: voxels of THIS shard; index_offset: global voxel index of its (0,0,0) (slab sharding:
 * world coordinates are always computed from the global index, so a slab is bit-identical to
 * the same voxels of an unsharded volume).  origin = f32(vol_bnds[:,0]) (grid_fusion.py:44),
 * trunc = 5 * voxel_size (grid_fusion.py:37). */
int tsdf_dense_create(const int64_t dims[3], const int64_t index_offset[3], const float origin[3],
                      double voxel_size, double trunc, int device, tsdf_dense_t** out);
/* Cyclic brick-column shard of a volume of global_dims voxels: shard s of n owns
 * the 8-voxel x-columns c with c % 2n in {s, 2n-1-s} (mirrored pairs), stored contiguously in
 * local x order, so every rank sees a similar share of each frame's frustum.  The shard's local dims are
 * (sum of its column widths, Y, Z); tsdf_dense_get/set use that local C-order.  n_shards = 1
 * is tsdf_dense_create with a zero offset.  Replaces the same constructor as above. */
int tsdf_dense_create_shard(const int64_t global_dims[3], int shard, int n_shards,
                            const float origin[3], double voxel_size, double trunc, int device,
                            tsdf_dense_t** out);
int tsdf_dense_destroy(tsdf_dense_t* h);
int tsdf_dense_reset(tsdf_dense_t* h); /* tsdf = 1, weight = 0, colour = 0 (grid_fusion.py:52-55) */

/* One frame: TSDFVolume.integrate(color_im, depth_im, cam_intr, cam_pose, obs_weight)
 * (grid_fusion.py:214-314).  K: the 3x3 intrinsics as given (row-major float64); the kernel uses
 * f64(f32(K)) like cam2pix (:190).  world_to_cam: np.linalg.inv(cam_pose) computed by the
 * caller (:265), row-major 4x4 float64.  Images: height, width < 2^24 and height*width < 2^28
 * (the gathers use 32-bit byte offsets), else TSDF_E_ARG. */
int tsdf_dense_integrate(tsdf_dense_t* h, const void* depth, int depth_kind, const void* color,
                         int color_kind, int height, int width, const double K[9],
                         const double world_to_cam[16], double obs_weight, int flags);

/* F frames back to back on the handle's stream (the bench's step).  depth/color point at F
 * consecutive frames (frame stride = H*W elements); world_to_cam: F*16 doubles (host);
 * obs_weight: F doubles (host) or NULL for all 1.0. */
int tsdf_dense_integrate_batch(tsdf_dense_t* h, int n_frames, const void* depth, int depth_kind,
                               const void* color, int color_kind, int height, int width,
                               const double K[9], const double* world_to_cam,
                               const double* obs_weight, int flags);

/* get_volume (grid_fusion.py:316-320) plus weight: C-order (X,Y,Z) float32 host arrays of
 * this shard; any pointer may be NULL to skip that field. */
int tsdf_dense_get(tsdf_dense_t* h, float* tsdf, float* weight, float* color);
int tsdf_dense_set(tsdf_dense_t* h, const float* tsdf, const float* weight, const float* color);
int tsdf_dense_sync(tsdf_dense_t* h);
/* Frames one launch integrates (the temporal batch: 32 in this build, 16 or 8 with -DTSDF_MAX_BATCH;
 * TSDF_BATCH overrides per process); calls of n frames run ceil(n / batch) + 2 pipelined launches. */
int tsdf_dense_frames_per_launch(tsdf_dense_t* h, int* n);
/* Mesh of the shard's tsdf at level 0 (get_mesh / get_point_cloud, grid_fusion.py:322-360; the
 * reference runs skimage's marching_cubes_lewiner on the host).  extract runs marching cubes on
 * the device and keeps the result in the handle; get_mesh copies it out: verts n_verts x 3 f32
 * world coordinates (index-space vertex * voxel_size + origin, in f32 like NumPy), normals
 * n_verts x 3 f32 unit (towards positive tsdf), colors n_verts x 3 uint8 r, g, b of the voxel at
 * round(vertex) (grid_fusion.py:336-346), faces n_tris x 3 int32 vertex ids.  One vertex per
 * grid edge whose end values straddle 0 (one below 0, one not), at the linear interpolation;
 * vertices ordered by (voxel, axis) in C-order and shared by the cells around the edge.  Any
 * output pointer may be NULL.  Vertex world x comes from the GLOBAL voxel index, so a slab
 * shard meshed alone gives the mesh of its own sub-volume in world coordinates; a cyclic column
 * shard needs its neighbours' border rows (tsdf_dense_extract_mesh_halo), else TSDF_E_ARG. */
int tsdf_dense_extract_mesh(tsdf_dense_t* h, int64_t* n_verts, int64_t* n_tris);
int tsdf_dense_get_mesh(tsdf_dense_t* h, float* verts, float* normals, uint8_t* colors, int32_t* faces);
/* Sharded marching cubes.  mesh_halo_rows: the global x rows (sorted) of the
 * unsharded volume (x extent global_x) that this shard's cells and gradients read but do not
 * own; with rows == NULL only *n_rows is set, else rows must hold *n_rows >= that many.
 * extract_mesh_halo: marching cubes over the cells anchored at the shard's own rows, given those
 * rows (halo_gx[n_halo] global x, halo_tsdf / halo_color n_halo x Y x Z C-order float32; host, or
 * device with TSDF_DEVICE_PTRS).  The shard's mesh holds its own cells' triangles and every
 * vertex they use, including copies of the next shard's border vertices; get_mesh_keys gives
 * each vertex's global identity ((x*Y + y)*Z + z)*3 + axis, the order of the unsharded mesh,
 * so the union of the shards' meshes, vertices merged by key, is the unsharded mesh. */
int tsdf_dense_mesh_halo_rows(tsdf_dense_t* h, int64_t global_x, int64_t* rows, int64_t* n_rows);
int tsdf_dense_extract_mesh_halo(tsdf_dense_t* h, int64_t global_x, const int64_t* halo_gx, int64_t n_halo,
                                 const float* halo_tsdf, const float* halo_color, int flags, int64_t* n_verts,
                                 int64_t* n_tris);
int tsdf_dense_get_mesh_keys(tsdf_dense_t* h, int64_t* keys);
/* Local x rows (rows[n_rows], local indices) of the shard in C-order (n_rows, Y, Z) float32 -- the
 * halo rows another shard needs and the rows of a device-side gather (get_volume of a sharded
 * volume).  Host pointers, or device pointers with TSDF_DEVICE_PTRS; NULL skips a field. */
int tsdf_dense_get_rows(tsdf_dense_t* h, const int64_t* rows, int64_t n_rows, float* tsdf, float* weight,
                        float* color, int flags);
/* The marching-cubes case table in use: tri[256][16] cube-edge ids (-1 padded; edge e joins the
 * corners differing in bit e / 4 of the corner index, its lower corner's other two bits being
 * e % 4 in increasing bit order), ntri[256] triangles per case.  Host-only; no device needed. */
int tsdf_mc_table(int8_t* tri, uint8_t* ntri);
int tsdf_dense_stats(tsdf_dense_t* h, tsdf_stats_t* out, int reset);
int tsdf_dense_set_profiling(tsdf_dense_t* h, int on);

/* ---- voxel hash: replaces HashTable (hash_fusion.py:29-507) --------------------------------
 * Keys are 8x8x8 voxel blocks.  `capacity` is the reference's map_size (hash_fusion.py:34): the
 * modulus of hash_function (hash_fusion.py:182-190, tsdf_hash_keys) and the size the 0.75
 * load-factor policy is kept against.  The device table has S = the power of two >= capacity
 * slots; the home slot of block (bx,by,bz) is the reference's hash of the block coordinates in
 * int64 (int_bits = 64, NumPy 2 / Linux) or wrapping int32 (int_bits = 32, the author's Windows
 * run), floor-mod S.  Open addressing, linear probe, lock-free CAS insert.  Shard s of n_shards
 * owns the blocks whose home slot (in the S of create) falls in [s*S/n, (s+1)*S/n). */
int tsdf_hash_create(const int64_t dims[3], const float origin[3], double voxel_size,
                     double trunc, int64_t capacity, int64_t max_blocks, int int_bits,
                     int shard, int n_shards, int device, tsdf_hash_t** out);
int tsdf_hash_destroy(tsdf_hash_t* h);
int tsdf_hash_reset(tsdf_hash_t* h);

/* HashTable.integrate (hash_fusion.py:103-145): same voxel set as the grid; obs_weight is
 * ignored (always 1) exactly like the reference (hash_fusion.py:141,145). */
int tsdf_hash_integrate(tsdf_hash_t* h, const void* depth, int depth_kind, const void* color,
                        int color_kind, int height, int width, const double K[9],
                        const double world_to_cam[16], int flags);
int tsdf_hash_integrate_batch(tsdf_hash_t* h, int n_frames, const void* depth, int depth_kind,
                              const void* color, int color_kind, int height, int width,
                              const double K[9], const double* world_to_cam, int flags);

/* Per-voxel entry API (get_hash_entry / add_hash_entry / remove, hash_fusion.py:199-393),
 * batched: ijk is n x 3 int64 voxel indices (host).
 *   lookup: found[i] = 1 and the voxel's (tsdf, weight, colour) if voxel i has an entry.
 *   insert: creates the entry (block allocated if needed); if tsdf/weight/color are non-NULL
 *           they set the voxel's values, else the voxel keeps (1, 0, 0).  slot[i] = table slot
 *           of the block, local[i] = voxel index inside the block (the reference returns
 *           (bucket, slot)).  Inserting an existing entry finds it (no duplicates).
 *   remove: removed[i] = 1 if the entry existed; a block whose last entry goes is freed. */
int tsdf_hash_lookup(tsdf_hash_t* h, const int64_t* ijk, int64_t n, float* tsdf, float* weight,
                     float* color, uint8_t* found);
int tsdf_hash_insert(tsdf_hash_t* h, const int64_t* ijk, int64_t n, const float* tsdf,
                     const float* weight, const float* color, int64_t* slot, int32_t* local);
int tsdf_hash_remove(tsdf_hash_t* h, const int64_t* ijk, int64_t n, uint8_t* removed);
/* double_table_size (hash_fusion.py:414-437): the table size becomes new_capacity (the device
 * table rehashes into the power of two >= it when that changes). */
int tsdf_hash_resize(tsdf_hash_t* h, int64_t new_capacity);
int tsdf_hash_info(tsdf_hash_t* h, tsdf_hash_info_t* out);
/* Sparse block transfer for merging bucket-range shards: only live blocks move.
 * export: with bxyz == NULL, *n_blocks = live blocks; else fills up to *n_blocks (must be >= the
 *   live count) blocks: bxyz n x 3 int32 block coordinates, tsdf/weight/color n x 512 float32 in
 *   brick-local order (x*8 + y)*8 + z, occ n x 8 uint64 voxel-entry words (word z, bit x*8+y);
 *   any field pointer may be NULL.  Host pointers, or device pointers with TSDF_DEVICE_PTRS.
 * import: find-or-insert each block (distinct, inside the volume) and overwrite its contents and
 *   entry words (NULL occ: every voxel has an entry).  The table / pool grow as needed. */
int tsdf_hash_export_blocks(tsdf_hash_t* h, int32_t* bxyz, float* tsdf, float* weight, float* color,
                            uint64_t* occ, int64_t* n_blocks, int flags);
int tsdf_hash_import_blocks(tsdf_hash_t* h, const int32_t* bxyz, int64_t n_blocks, const float* tsdf,
                            const float* weight, const float* color, const uint64_t* occ, int flags);
/* get_volume (hash_fusion.py:442-463): densify into C-order (X,Y,Z) host arrays; voxels
 * without an entry get tsdf 1, weight 0, colour 0.  Any pointer may be NULL. */
int tsdf_hash_get_dense(tsdf_hash_t* h, float* tsdf, float* weight, float* color);
/* The same densify on the device, into a dense handle of the hash's dims (unsharded; it is reset
 * first): get_mesh / get_point_cloud of the hash (hash_fusion.py:465-507) then run the dense
 * handle's marching cubes without a host round trip of the volume. */
int tsdf_hash_to_dense(tsdf_hash_t* h, tsdf_dense_t* d);
int tsdf_hash_sync(tsdf_hash_t* h);
/* sync, then a pool on mapped memory hands the memory above its live blocks back (pool_capacity
 * = live blocks + ~3 %, in whole 8 MB pieces; the live blocks move into fresh mapped ranges by one
 * device copy): the end of an asynchronous run, whose growth had to stay ahead of the launches in
 * flight.  get_volume / get_mesh call it.  Not in the reference (its pool is a Python dict). */
int tsdf_hash_trim(tsdf_hash_t* h);
int tsdf_hash_stats(tsdf_hash_t* h, tsdf_stats_t* out, int reset);
int tsdf_hash_set_profiling(tsdf_hash_t* h, int on);
/* Frames one launch of this table integrates (as tsdf_dense_frames_per_launch: 32 in this build;
 * shards of n_shards > 1 always kMaxBatch). */
int tsdf_hash_frames_per_launch(tsdf_hash_t* h, int* n);

/* ---- frame utilities ---------------------------------------------------------------------
 * Volume bounds from view frustums: the demo loop grid_demo1.py:50-64 (hash_demo1.py:93-107)
 * over get_view_frustum (grid_fusion.py:371-383).  For each of
 * n_frames depth images (H*W each, kind U16_MM or F64_M; host, or device with TSDF_DEVICE_PTRS;
 * TSDF_DEPTH_INVALID_65535 masks 65535 mm; on HIP device `device`): the image's max depth, the 5 frustum points
 * transformed by cam_pose (n_frames*16 doubles, camera-to-world, host), then
 * bounds[2r] = min(bounds[2r], min over points), bounds[2r+1] = max(...) for r = x, y, z
 * (bounds is in/out: the demo starts from zeros).  Optional outputs: max_depth (n_frames
 * doubles, metres) and frustum_pts (n_frames x 3 x 5 doubles, get_view_frustum's array).
 * All values equal the reference's f64 results bit for bit. */
int tsdf_frustum_bounds(const void* depth, int depth_kind, int n_frames, int height, int width,
                        const double K[9], const double* cam_poses, int flags, int device,
                        double* max_depth, double* frustum_pts, double bounds[6]);

/* hash_function over n coordinate triples (host in, host out), computed on the device.  The
 * same arithmetic as the kernels' home-slot computation. */
int tsdf_hash_keys(const int64_t* xyz, int64_t n, int64_t table_size, int int_bits,
                   int64_t* out, int device);

#ifdef __cplusplus
}
#endif
#endif /* TSDF_HIP_H */
