// tsdf_mesh.hip -- mesh / point-cloud extraction from a dense volume: the
// MI355X replacement of get_mesh / get_point_cloud (grid_fusion.py:322-360), which run
// skimage.measure.marching_cubes_lewiner on the host.
//
// Marching cubes at level 0 over the handle's brick layout, in three passes:
//   k_mc_classify  one thread per voxel (C-order): the voxel's three +axis grid edges that cross
//                  0 (a vertex each) and, for voxels that anchor a cell, the cell's case and
//                  triangle count;
//   (exclusive scans of both counts: vertex and triangle offsets, in C-order)
//   k_mc_vertices  one thread per voxel with crossings: vertex position (linear interpolation,
//                  index space, then world = p * voxel_size + origin in f32 as NumPy does),
//                  normal (interpolated central-difference gradient, pointing to positive tsdf)
//                  and colour (grid_fusion.py:336-346: the voxel at round(p), decoded);
//   k_mc_triangles one thread per cell: the case's triangles, each cube edge mapped to the
//                  global vertex id of its grid edge.
// Vertices are ordered by (voxel, axis) in C-order and shared between cells (an indexed mesh
// like skimage's); the case table comes from one rule (tsdf_mc_table, oracle/mc_table.py).
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <vector>

#include "tsdf_host.h"

using namespace tsdf;

namespace {

// ---- case table (the rule of oracle/mc_table.py) ------------------------------------------------
struct McTable {
    signed char tri[256][16];  // edge ids, -1 padded
    unsigned char ntri[256];
};

McTable build_table() {
    McTable t;
    std::memset(t.tri, -1, sizeof(t.tri));
    int edge_of[8][8];
    int corner_pair[12][2];
    int ne = 0;
    for (int a = 0; a < 8; ++a)
        for (int b = 0; b < 8; ++b) edge_of[a][b] = -1;
    for (int axis = 0; axis < 3; ++axis)
        for (int c = 0; c < 8; ++c)
            if (!((c >> axis) & 1)) {
                corner_pair[ne][0] = c;
                corner_pair[ne][1] = c | (1 << axis);
                edge_of[c][c | (1 << axis)] = edge_of[c | (1 << axis)][c] = ne;
                ++ne;
            }
    int faces[6][4];
    int nf = 0;
    for (int axis = 0; axis < 3; ++axis) {
        const int u = (axis + 1) % 3, v = (axis + 2) % 3;
        for (int side = 0; side < 2; ++side) {
            const int base = side << axis;
            int cyc[4] = {base, base | (1 << u), base | (1 << u) | (1 << v), base | (1 << v)};
            if (side == 0) std::swap(cyc[0], cyc[3]), std::swap(cyc[1], cyc[2]);  // reverse: CCW from outside
            for (int i = 0; i < 4; ++i) faces[nf][i] = cyc[i];
            ++nf;
        }
    }
    for (int cfg = 0; cfg < 256; ++cfg) {
        int seg[12];
        for (int i = 0; i < 12; ++i) seg[i] = -1;
        auto in = [&](int c) { return (cfg >> c) & 1; };
        for (int f = 0; f < 6; ++f) {
            const int* cyc = faces[f];
            int n_in = 0;
            for (int i = 0; i < 4; ++i) n_in += in(cyc[i]);
            if (n_in == 0 || n_in == 4) continue;
            for (int i = 0; i < 4; ++i) {
                const int a = cyc[i], b = cyc[(i + 1) % 4];
                if (in(a) && !in(b)) {  // the walk leaves a run of inside corners at edge (a, b)
                    int j = i;
                    while (in(cyc[(j + 3) % 4])) j = (j + 3) % 4;
                    const int p = cyc[(j + 3) % 4], q = cyc[j];  // where the run was entered
                    seg[edge_of[a][b]] = edge_of[p][q];
                }
            }
        }
        int k = 0;
        bool left[12];
        for (int i = 0; i < 12; ++i) left[i] = seg[i] >= 0;
        for (int start = 0; start < 12; ++start) {
            if (!left[start]) continue;
            int loop[12], n = 0;
            int e = start;
            do {
                loop[n++] = e;
                left[e] = false;
                e = seg[e];
            } while (e != start);
            for (int i = 1; i + 1 < n; ++i) {
                t.tri[cfg][k++] = (signed char)loop[0];
                t.tri[cfg][k++] = (signed char)loop[i];
                t.tri[cfg][k++] = (signed char)loop[i + 1];
            }
        }
        t.ntri[cfg] = (unsigned char)(k / 3);
    }
    return t;
}

const McTable& table() {
    static const McTable t = build_table();
    return t;
}

// cube edge e -> (corner offset bits of its lower corner, axis); edges are sorted by axis
__device__ inline void edge_anchor(int e, int& off, int& axis) {
    axis = e >> 2;
    const int r = e & 3;  // the two other coordinate bits, in increasing bit order
    const int u = axis == 0 ? 1 : 0, v = axis == 2 ? 1 : 2;
    off = ((r & 1) << u) | (((r >> 1) & 1) << v);
}

// The volume as marching cubes sees it: rows of constant global x.  Local rows live in the
// handle's brick pool; rows owned by other shards (halo rows, exchanged by the caller) arrive as
// C-order (Y, Z) slices.  row_map[gx - xlo] says where global row gx is: >= 0 local row,
// <= -2 halo row -2-r, -1 absent.  Marching cubes runs over the global x range [xlo, xhi):
// gradients clamp there, x-edges and cells need gx + 1 < xhi.  A shard's "vertex rows" are its
// local rows plus each cap row (a halo row gx whose gx - 1 is local): the cells a shard owns are
// those anchored at its local rows, and a cap row carries the y/z-edge vertices of their +x faces
// (duplicates of the next shard's own vertices, identified by the same global key).
struct Grid {
    int Y, Z;
    int xlo, xhi;
    int nby, nbz;              // brick geometry of the local rows
    const int* row_map;        // [xhi - xlo]
    const int* vrow_gx;        // [nrows] global x of the vertex rows, increasing
    const unsigned char* vrow_cap;  // [nrows] 1: cap row (y/z-edge vertices only, no cells)
    const float* t;            // brick-layout state (local rows)
    const float* c;
    const float* ht;           // halo rows, C-order [n_halo][Y][Z]
    const float* hc;
};

__device__ inline float gval(const Grid& g, const float* brick, const float* halo, int gx, int y, int z) {
    const int r = g.row_map[gx - g.xlo];
    if (r >= 0) {
        const size_t b = ((size_t)(r >> 3) * g.nby + (y >> 3)) * g.nbz + (z >> 3);
        return brick[b * kBrickVox + (size_t)(((r & 7) * 8 + (y & 7)) * 8 + (z & 7))];
    }
    return halo[((size_t)(-2 - r) * g.Y + y) * g.Z + z];
}
__device__ inline float tval(const Grid& g, int gx, int y, int z) { return gval(g, g.t, g.ht, gx, y, z); }
__device__ inline float cval(const Grid& g, int gx, int y, int z) { return gval(g, g.c, g.hc, gx, y, z); }

__global__ void k_mc_classify(Grid g, int nrows, const unsigned char* __restrict__ ntri,
                              unsigned char* __restrict__ ebits, unsigned char* __restrict__ cubes,
                              unsigned* __restrict__ vcnt, unsigned* __restrict__ tcnt) {
    const size_t n = (size_t)nrows * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), row = (int)(xy / g.Y);
        const int x = g.vrow_gx[row];
        const bool cap = g.vrow_cap[row] != 0;
        const bool in0 = tval(g, x, y, z) < 0.0f;
        const bool xn = !cap && x + 1 < g.xhi;  // x-edge and cells only from local rows
        unsigned bits = 0;
        if (xn && (tval(g, x + 1, y, z) < 0.0f) != in0) bits |= 1u;
        if (y + 1 < g.Y && (tval(g, x, y + 1, z) < 0.0f) != in0) bits |= 2u;
        if (z + 1 < g.Z && (tval(g, x, y, z + 1) < 0.0f) != in0) bits |= 4u;
        unsigned cube = 0, nt = 0;
        if (xn && y + 1 < g.Y && z + 1 < g.Z) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
                cube |= (unsigned)(tval(g, x + (c & 1), y + ((c >> 1) & 1), z + ((c >> 2) & 1)) < 0.0f) << c;
            nt = ntri[cube];
        }
        ebits[i] = (unsigned char)bits;
        cubes[i] = (unsigned char)cube;
        vcnt[i] = (unsigned)__popc(bits);
        tcnt[i] = nt;
    }
}

// central-difference gradient of the tsdf at a voxel (indices clamped at the faces of the
// meshed range)
__device__ inline void grad(const Grid& g, int x, int y, int z, float out[3]) {
    out[0] = tval(g, min(x + 1, g.xhi - 1), y, z) - tval(g, max(x - 1, g.xlo), y, z);
    out[1] = tval(g, x, min(y + 1, g.Y - 1), z) - tval(g, x, max(y - 1, 0), z);
    out[2] = tval(g, x, y, min(z + 1, g.Z - 1)) - tval(g, x, y, max(z - 1, 0));
}

__global__ void k_mc_vertices(Grid g, int nrows, const unsigned char* __restrict__ ebits,
                              const unsigned* __restrict__ vbase, float ox, float oy, float oz, float vs,
                              float* __restrict__ verts, float* __restrict__ normals,
                              unsigned char* __restrict__ colors, long long* __restrict__ keys) {
    const size_t n = (size_t)nrows * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned bits = ebits[i];
        if (!bits) continue;
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), x = g.vrow_gx[xy / g.Y];
        const float v1 = tval(g, x, y, z);
        float g1[3];
        grad(g, x, y, z, g1);
        unsigned id = vbase[i];
        for (int a = 0; a < 3; ++a) {
            if (!((bits >> a) & 1u)) continue;
            const int x2 = x + (a == 0), y2 = y + (a == 1), z2 = z + (a == 2);
            const float v2 = tval(g, x2, y2, z2);
            const float t = (0.0f - v1) / (v2 - v1);
            float p[3] = {(float)x, (float)y, (float)z};
            p[a] = p[a] + t;
            float g2[3];
            grad(g, x2, y2, z2, g2);
            float nrm[3];
            for (int k = 0; k < 3; ++k) nrm[k] = g1[k] + t * (g2[k] - g1[k]);
            const float len = __fsqrt_rn(nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2]);
            const float o[3] = {ox, oy, oz};
            for (int k = 0; k < 3; ++k) {
                verts[3 * (size_t)id + k] = p[k] * vs + o[k];  // verts * voxel_size + origin (f32)
                normals[3 * (size_t)id + k] = len > 0.0f ? nrm[k] / len : 0.0f;
            }
            // grid_fusion.py:336-346: colour of the voxel at round(verts), decoded to uint8
            const int rx = (int)rintf(p[0]), ry = (int)rintf(p[1]), rz = (int)rintf(p[2]);
            const float cv = cval(g, rx, ry, rz);
            const float cb = floorf(cv / 65536.0f);
            const float cg = floorf((cv - cb * 65536.0f) / 256.0f);
            const float cr = cv - cb * 65536.0f - cg * 256.0f;
            colors[3 * (size_t)id + 0] = (unsigned char)(int)floorf(cr);
            colors[3 * (size_t)id + 1] = (unsigned char)(int)floorf(cg);
            colors[3 * (size_t)id + 2] = (unsigned char)(int)floorf(cb);
            // global identity of the vertex: (voxel, axis) in the unsharded volume's C-order
            keys[id] = ((((long long)x * g.Y) + y) * g.Z + z) * 3 + a;
            ++id;
        }
    }
}

__global__ void k_mc_triangles(Grid g, int nrows, const signed char* __restrict__ tri,
                               const unsigned char* __restrict__ cubes, const unsigned char* __restrict__ ebits,
                               const unsigned* __restrict__ vbase, const unsigned* __restrict__ tbase,
                               int* __restrict__ faces) {
    const size_t n = (size_t)nrows * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned cube = cubes[i];
        if (cube == 0 || cube == 255) continue;
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), row = (int)(xy / g.Y);
        size_t f = tbase[i];
        const signed char* rowt = tri + 16 * cube;
        for (int k = 0; rowt[k] >= 0; k += 3) {
            int vid[3];
            for (int j = 0; j < 3; ++j) {
                int off, axis;
                edge_anchor(rowt[k + j], off, axis);
                // the vertex row after a local row is global x + 1 (local or cap)
                const size_t e = (((size_t)(row + (off & 1)) * g.Y + (y + ((off >> 1) & 1))) * g.Z) +
                                 (z + ((off >> 2) & 1));
                const unsigned bits = ebits[e];
                vid[j] = (int)(vbase[e] + (unsigned)__popc(bits & ((1u << axis) - 1u)));
            }
            // the table's loops wind around the inside corners; emit (0, 2, 1) so the face
            // normal points to positive tsdf, like the vertex normals
            faces[3 * f + 0] = vid[0];
            faces[3 * f + 1] = vid[2];
            faces[3 * f + 2] = vid[1];
            ++f;
        }
    }
}

template <typename T>
int dev_alloc(T** p, size_t n) {
    TSDF_HIP(hipMalloc((void**)p, sizeof(T) * (n ? n : 1)));
    return TSDF_OK;
}

}  // namespace

namespace tsdf {

void Mesh::release() {
    for (void* p : {(void*)verts, (void*)normals, (void*)colors, (void*)faces, (void*)keys})
        if (p) (void)hipFree(p);
    verts = normals = nullptr;
    colors = nullptr;
    faces = nullptr;
    keys = nullptr;
    n_verts = n_tris = 0;
}

int mesh_domain(const Vol& v, long long global_x, const int64_t* halo_gx, long long n_halo, MeshDomain* d) {
    const int nl = v.dims[0];
    auto gx_of = [&](int lr) { return v.off[0] + col_gx(v, lr >> 3) + (lr & 7); };
    if (global_x > 0) {
        d->xlo = 0;
        d->xhi = (int)global_x;
    } else {  // the shard alone: its own rows must be contiguous
        if (v.xstride != kBrickEdge && v.nb[0] > 1)
            return set_error(TSDF_E_ARG, "a cyclic column shard is meshed with its neighbours' border rows "
                                         "(tsdf_dense_extract_mesh_halo)");
        d->xlo = gx_of(0);
        d->xhi = gx_of(nl - 1) + 1;
    }
    const int span = d->xhi - d->xlo;
    if (span <= 0 || global_x > (1 << 24)) return set_error(TSDF_E_ARG, "bad global x extent %lld", global_x);
    d->row_map.assign(span, -1);
    for (int lr = 0; lr < nl; ++lr) {
        const int gx = gx_of(lr);
        if (gx < d->xlo || gx >= d->xhi) return set_error(TSDF_E_ARG, "local row %d (x %d) outside [%d, %d)", lr, gx, d->xlo, d->xhi);
        d->row_map[gx - d->xlo] = lr;
    }
    for (long long h = 0; h < n_halo; ++h) {
        const long long gx = halo_gx[h];
        if (gx < d->xlo || gx >= d->xhi) return set_error(TSDF_E_ARG, "halo row %lld outside [%d, %d)", gx, d->xlo, d->xhi);
        if (d->row_map[gx - d->xlo] >= 0) return set_error(TSDF_E_ARG, "halo row %lld is a local row", gx);
        if (d->row_map[gx - d->xlo] <= -2) return set_error(TSDF_E_ARG, "halo row %lld given twice", gx);
        d->row_map[gx - d->xlo] = (int)(-2 - h);
    }
    auto present = [&](long long gx) { return gx < d->xlo || gx >= d->xhi || d->row_map[gx - d->xlo] != -1; };
    d->vrow_gx.clear();
    d->vrow_cap.clear();
    for (int gx = d->xlo; gx < d->xhi; ++gx) {
        const int r = d->row_map[gx - d->xlo];
        const bool local = r >= 0, prev_local = gx > d->xlo && d->row_map[gx - 1 - d->xlo] >= 0;
        if (!local && !prev_local) continue;
        // every row the cells and gradients read: x - 1, x + 1 (and x + 1 of a cap row)
        if (!present(gx) || !present(gx - 1) || !present(gx + 1))
            return set_error(TSDF_E_ARG, "mesh of x row %d needs rows %d..%d: pass the missing border rows "
                                         "(tsdf_dense_mesh_halo_rows)", gx, gx - 1, gx + 1);
        d->vrow_gx.push_back(gx);
        d->vrow_cap.push_back(local ? 0 : 1);
    }
    return TSDF_OK;
}

int mesh_halo_rows(const Vol& v, long long global_x, std::vector<long long>* out) {
    out->clear();
    if (global_x <= 0 || global_x > (1 << 24)) return set_error(TSDF_E_ARG, "bad global x extent %lld", global_x);
    std::vector<char> local((size_t)global_x, 0);
    for (int lr = 0; lr < v.dims[0]; ++lr) {
        const long long gx = v.off[0] + (long long)col_gx(v, lr >> 3) + (lr & 7);
        if (gx >= global_x) return set_error(TSDF_E_ARG, "local row at x %lld beyond the global extent", gx);
        local[gx] = 1;
    }
    std::vector<char> need((size_t)global_x, 0);
    for (long long gx = 0; gx < global_x; ++gx) {
        if (!local[gx]) continue;
        if (gx - 1 >= 0) need[gx - 1] = 1;
        if (gx + 1 < global_x) need[gx + 1] = 1;
        if (gx + 2 < global_x && !local[gx + 1]) need[gx + 2] = 1;  // gradient of the cap row
    }
    for (long long gx = 0; gx < global_x; ++gx)
        if (need[gx] && !local[gx]) out->push_back(gx);
    return TSDF_OK;
}

// Extract into m (device buffers): the cells anchored at the shard's local rows over the range
// and halo rows of `d` (halo rows: device C-order slices, nullptr when there are none).
int extract_mesh(Base& B, const Pool& pool, Mesh& m, const MeshDomain& d, const float* ht, const float* hc) {
    m.release();
    const McTable& tab = table();
    const int nrows = (int)d.vrow_gx.size();
    Grid g;
    g.Y = B.vol.dims[1];
    g.Z = B.vol.dims[2];
    g.xlo = d.xlo;
    g.xhi = d.xhi;
    g.nby = B.vol.nb[1];
    g.nbz = B.vol.nb[2];
    g.t = pool.tsdf;
    g.c = pool.color;
    g.ht = ht;
    g.hc = hc;
    const size_t n = (size_t)nrows * g.Y * g.Z;
    if (n >= (1ull << 31)) return set_error(TSDF_E_ARG, "volume too large for one mesh extraction (>= 2^31 voxels)");
    hipStream_t s = B.stream;
    unsigned char *ebits = nullptr, *cubes = nullptr, *ntri = nullptr, *vcap = nullptr;
    signed char* dtri = nullptr;
    unsigned *vcnt = nullptr, *tcnt = nullptr, *vbase = nullptr, *tbase = nullptr;
    int *rmap = nullptr, *vgx = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int r = TSDF_OK;
    auto cleanup = [&]() {
        for (void* p : {(void*)ebits, (void*)cubes, (void*)ntri, (void*)dtri, (void*)vcnt, (void*)tcnt, (void*)vbase,
                        (void*)tbase, (void*)rmap, (void*)vgx, (void*)vcap, tmp})
            if (p) (void)hipFree(p);
    };
    do {
        if ((r = dev_alloc(&ebits, n)) || (r = dev_alloc(&cubes, n)) || (r = dev_alloc(&ntri, 256)) ||
            (r = dev_alloc(&dtri, 256 * 16)) || (r = dev_alloc(&vcnt, n)) || (r = dev_alloc(&tcnt, n)) ||
            (r = dev_alloc(&vbase, n + 1)) || (r = dev_alloc(&tbase, n + 1)) ||
            (r = dev_alloc(&rmap, d.row_map.size())) || (r = dev_alloc(&vgx, (size_t)nrows)) ||
            (r = dev_alloc(&vcap, (size_t)nrows)))
            break;
        hipError_t e = hipMemcpyAsync(ntri, tab.ntri, 256, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(dtri, tab.tri, 256 * 16, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(rmap, d.row_map.data(), sizeof(int) * d.row_map.size(), hipMemcpyHostToDevice, s);
        if (e == hipSuccess && nrows) e = hipMemcpyAsync(vgx, d.vrow_gx.data(), sizeof(int) * nrows, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && nrows) e = hipMemcpyAsync(vcap, d.vrow_cap.data(), nrows, hipMemcpyHostToDevice, s);
        g.row_map = rmap;
        g.vrow_gx = vgx;
        g.vrow_cap = vcap;
        if (n == 0) {
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) r = set_error(TSDF_E_HIP, "mesh setup: %s", hipGetErrorString(e));
            break;
        }
        const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, (size_t)B.n_cu * 32);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_mc_classify, dim3(grid), dim3(256), 0, s, g, nrows, (const unsigned char*)ntri, ebits,
                               cubes, vcnt, tcnt);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, vcnt, vbase, (int)n, s);
        if (e == hipSuccess) e = hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1);
        if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, vcnt, vbase, (int)n, s);
        if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, tcnt, tbase, (int)n, s);
        unsigned last[4] = {0, 0, 0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(&last[0], vbase + n - 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&last[1], vcnt + n - 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&last[2], tbase + n - 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&last[3], tcnt + n - 1, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            r = set_error(TSDF_E_HIP, "mesh classify/scan: %s", hipGetErrorString(e));
            break;
        }
        m.n_verts = (long long)last[0] + last[1];
        m.n_tris = (long long)last[2] + last[3];
        if ((r = dev_alloc(&m.verts, 3 * m.n_verts)) || (r = dev_alloc(&m.normals, 3 * m.n_verts)) ||
            (r = dev_alloc(&m.colors, 3 * m.n_verts)) || (r = dev_alloc(&m.faces, 3 * m.n_tris)) ||
            (r = dev_alloc(&m.keys, m.n_verts)))
            break;
        hipLaunchKernelGGL(k_mc_vertices, dim3(grid), dim3(256), 0, s, g, nrows, (const unsigned char*)ebits,
                           (const unsigned*)vbase, B.vol.origin[0], B.vol.origin[1], B.vol.origin[2],
                           (float)B.vol.vs, m.verts, m.normals, m.colors, m.keys);
        hipLaunchKernelGGL(k_mc_triangles, dim3(grid), dim3(256), 0, s, g, nrows, (const signed char*)dtri,
                           (const unsigned char*)cubes, (const unsigned char*)ebits, (const unsigned*)vbase,
                           (const unsigned*)tbase, m.faces);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) r = set_error(TSDF_E_HIP, "mesh emit: %s", hipGetErrorString(e));
    } while (false);
    cleanup();
    if (r != TSDF_OK) m.release();
    return r;
}

int copy_mesh(Base& B, const Mesh& m, float* verts, float* normals, uint8_t* colors, int32_t* faces,
              int64_t* keys) {
    hipStream_t s = B.stream;
    if (keys) TSDF_HIP(hipMemcpyAsync(keys, m.keys, sizeof(long long) * m.n_verts, hipMemcpyDeviceToHost, s));
    if (verts) TSDF_HIP(hipMemcpyAsync(verts, m.verts, sizeof(float) * 3 * m.n_verts, hipMemcpyDeviceToHost, s));
    if (normals) TSDF_HIP(hipMemcpyAsync(normals, m.normals, sizeof(float) * 3 * m.n_verts, hipMemcpyDeviceToHost, s));
    if (colors) TSDF_HIP(hipMemcpyAsync(colors, m.colors, 3 * m.n_verts, hipMemcpyDeviceToHost, s));
    if (faces) TSDF_HIP(hipMemcpyAsync(faces, m.faces, sizeof(int) * 3 * m.n_tris, hipMemcpyDeviceToHost, s));
    TSDF_HIP(hipStreamSynchronize(s));
    return TSDF_OK;
}

}  // namespace tsdf

extern "C" int tsdf_mc_table(int8_t* out, uint8_t* ntri) {
    if (!out) return set_error(TSDF_E_ARG, "null pointer");
    const McTable& t = table();
    std::memcpy(out, t.tri, sizeof(t.tri));
    if (ntri) std::memcpy(ntri, t.ntri, sizeof(t.ntri));
    return TSDF_OK;
}
