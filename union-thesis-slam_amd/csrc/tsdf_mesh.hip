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

struct Grid {
    int X, Y, Z;       // local voxels
    int nby, nbz;      // bricks per axis (y, z)
    const float* t;    // brick-layout state
    const float* c;
};

__device__ inline size_t brick_addr(const Grid& g, int x, int y, int z) {
    const size_t b = ((size_t)(x >> 3) * g.nby + (y >> 3)) * g.nbz + (z >> 3);
    return b * kBrickVox + (size_t)(((x & 7) * 8 + (y & 7)) * 8 + (z & 7));
}
__device__ inline float tval(const Grid& g, int x, int y, int z) { return g.t[brick_addr(g, x, y, z)]; }

__global__ void k_mc_classify(Grid g, const unsigned char* __restrict__ ntri, unsigned char* __restrict__ ebits,
                              unsigned char* __restrict__ cubes, unsigned* __restrict__ vcnt,
                              unsigned* __restrict__ tcnt) {
    const size_t n = (size_t)g.X * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), x = (int)(xy / g.Y);
        const bool in0 = tval(g, x, y, z) < 0.0f;
        unsigned bits = 0;
        if (x + 1 < g.X && (tval(g, x + 1, y, z) < 0.0f) != in0) bits |= 1u;
        if (y + 1 < g.Y && (tval(g, x, y + 1, z) < 0.0f) != in0) bits |= 2u;
        if (z + 1 < g.Z && (tval(g, x, y, z + 1) < 0.0f) != in0) bits |= 4u;
        unsigned cube = 0, nt = 0;
        if (x + 1 < g.X && y + 1 < g.Y && z + 1 < g.Z) {
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

// central-difference gradient of the tsdf at a voxel (indices clamped at the volume's faces)
__device__ inline void grad(const Grid& g, int x, int y, int z, float out[3]) {
    out[0] = tval(g, min(x + 1, g.X - 1), y, z) - tval(g, max(x - 1, 0), y, z);
    out[1] = tval(g, x, min(y + 1, g.Y - 1), z) - tval(g, x, max(y - 1, 0), z);
    out[2] = tval(g, x, y, min(z + 1, g.Z - 1)) - tval(g, x, y, max(z - 1, 0));
}

__global__ void k_mc_vertices(Grid g, const unsigned char* __restrict__ ebits, const unsigned* __restrict__ vbase,
                              float ox, float oy, float oz, float vs, float* __restrict__ verts,
                              float* __restrict__ normals, unsigned char* __restrict__ colors) {
    const size_t n = (size_t)g.X * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned bits = ebits[i];
        if (!bits) continue;
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), x = (int)(xy / g.Y);
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
            const float cv = g.c[brick_addr(g, rx, ry, rz)];
            const float cb = floorf(cv / 65536.0f);
            const float cg = floorf((cv - cb * 65536.0f) / 256.0f);
            const float cr = cv - cb * 65536.0f - cg * 256.0f;
            colors[3 * (size_t)id + 0] = (unsigned char)(int)floorf(cr);
            colors[3 * (size_t)id + 1] = (unsigned char)(int)floorf(cg);
            colors[3 * (size_t)id + 2] = (unsigned char)(int)floorf(cb);
            ++id;
        }
    }
}

__global__ void k_mc_triangles(Grid g, const signed char* __restrict__ tri, const unsigned char* __restrict__ cubes,
                               const unsigned char* __restrict__ ebits, const unsigned* __restrict__ vbase,
                               const unsigned* __restrict__ tbase, int* __restrict__ faces) {
    const size_t n = (size_t)g.X * g.Y * g.Z;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned cube = cubes[i];
        if (cube == 0 || cube == 255) continue;
        const int z = (int)(i % g.Z);
        const size_t xy = i / g.Z;
        const int y = (int)(xy % g.Y), x = (int)(xy / g.Y);
        size_t f = tbase[i];
        const signed char* row = tri + 16 * cube;
        for (int k = 0; row[k] >= 0; k += 3) {
            int vid[3];
            for (int j = 0; j < 3; ++j) {
                int off, axis;
                edge_anchor(row[k + j], off, axis);
                const size_t e = (((size_t)(x + (off & 1)) * g.Y + (y + ((off >> 1) & 1))) * g.Z) + (z + ((off >> 2) & 1));
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
    for (void* p : {(void*)verts, (void*)normals, (void*)colors, (void*)faces})
        if (p) (void)hipFree(p);
    verts = normals = nullptr;
    colors = nullptr;
    faces = nullptr;
    n_verts = n_tris = 0;
}

// Extract into m (device buffers) from a brick-layout volume of local dims X, Y, Z.
int extract_mesh(Base& B, const Pool& pool, Mesh& m) {
    m.release();
    const McTable& tab = table();
    Grid g;
    g.X = B.vol.dims[0];
    g.Y = B.vol.dims[1];
    g.Z = B.vol.dims[2];
    g.nby = B.vol.nb[1];
    g.nbz = B.vol.nb[2];
    g.t = pool.tsdf;
    g.c = pool.color;
    const size_t n = (size_t)g.X * g.Y * g.Z;
    if (n >= (1ull << 31)) return set_error(TSDF_E_ARG, "volume too large for one mesh extraction (>= 2^31 voxels)");
    hipStream_t s = B.stream;
    unsigned char *ebits = nullptr, *cubes = nullptr, *ntri = nullptr;
    signed char* dtri = nullptr;
    unsigned *vcnt = nullptr, *tcnt = nullptr, *vbase = nullptr, *tbase = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int r = TSDF_OK;
    auto cleanup = [&]() {
        for (void* p : {(void*)ebits, (void*)cubes, (void*)ntri, (void*)dtri, (void*)vcnt, (void*)tcnt, (void*)vbase,
                        (void*)tbase, tmp})
            if (p) (void)hipFree(p);
    };
    do {
        if ((r = dev_alloc(&ebits, n)) || (r = dev_alloc(&cubes, n)) || (r = dev_alloc(&ntri, 256)) ||
            (r = dev_alloc(&dtri, 256 * 16)) || (r = dev_alloc(&vcnt, n)) || (r = dev_alloc(&tcnt, n)) ||
            (r = dev_alloc(&vbase, n + 1)) || (r = dev_alloc(&tbase, n + 1)))
            break;
        hipError_t e = hipMemcpyAsync(ntri, tab.ntri, 256, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(dtri, tab.tri, 256 * 16, hipMemcpyHostToDevice, s);
        const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, (size_t)B.n_cu * 32);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_mc_classify, dim3(grid), dim3(256), 0, s, g, (const unsigned char*)ntri, ebits, cubes,
                               vcnt, tcnt);
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
            (r = dev_alloc(&m.colors, 3 * m.n_verts)) || (r = dev_alloc(&m.faces, 3 * m.n_tris)))
            break;
        hipLaunchKernelGGL(k_mc_vertices, dim3(grid), dim3(256), 0, s, g, (const unsigned char*)ebits,
                           (const unsigned*)vbase, B.vol.origin[0], B.vol.origin[1], B.vol.origin[2],
                           (float)B.vol.vs, m.verts, m.normals, m.colors);
        hipLaunchKernelGGL(k_mc_triangles, dim3(grid), dim3(256), 0, s, g, (const signed char*)dtri,
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

int copy_mesh(Base& B, const Mesh& m, float* verts, float* normals, uint8_t* colors, int32_t* faces) {
    hipStream_t s = B.stream;
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
