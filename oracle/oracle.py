"""TEST INFRASTRUCTURE ONLY -- the CPU checker for the TSDF fusion hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product (union-thesis-slam_amd/tsdf_amd) never does: it runs on its HIP library or fails.

Parity status: PINNED against golden vectors generated from the reference itself
(tools/gen_golden.py -> tests/golden/) and the author's recorded counts.

Contents
  * ctypes front-end of tsdf_oracle.c (exact scalar restatement, see that file's header);
  * OracleTSDFVolume / OracleHashVolume: the reference's constructor semantics
    (grid_fusion.py:22-55, hash_fusion.py:34-69) around the C integrate;
  * numpy_port_integrate / NumpyPortHash: NumPy restatements with the reference's own structure
    (full-volume vox2world -> np.dot rigid transform -> cam2pix -> masks -> gather/scatter,
    grid_fusion.py:260-314; the per-voxel hash loop, hash_fusion.py:134-145) -- bench.py's timed
    CPU baseline, pinned against the reference fixtures by tests/test_oracle_golden.py;
  * hash_keys: hash_function (hash_fusion.py:182-190) in int64 or wrapping-int32 mode.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P1, P2, P3 = 73856093, 19349669, 83492791


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "libtsdf_oracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libtsdf_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.oracle_dense_integrate.restype = ctypes.c_int64
        L.oracle_dense_integrate.argtypes = [P, P, ctypes.c_double, ctypes.c_double, P, P, P, P,
                                             P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_double, P]
        L.oracle_dense_integrate_slab.restype = ctypes.c_int64
        L.oracle_dense_integrate_slab.argtypes = [P, P, P, ctypes.c_double, ctypes.c_double, P, P, P,
                                                  P, P, ctypes.c_int, ctypes.c_int, P, P,
                                                  ctypes.c_double, P]
        L.oracle_dense_integrate_rows.restype = ctypes.c_int64
        L.oracle_dense_integrate_rows.argtypes = [P, P, P, P, ctypes.c_double, ctypes.c_double, P, P,
                                                  P, P, P, ctypes.c_int, ctypes.c_int, P, P,
                                                  ctypes.c_double, P]
        L.oracle_hash_integrate.restype = ctypes.c_int64
        L.oracle_hash_integrate.argtypes = [P, P, ctypes.c_double, ctypes.c_double, P, P, P, P,
                                            P, ctypes.c_int, ctypes.c_int, P, P, P, P]
        L.oracle_view_frustum.restype = None
        L.oracle_view_frustum.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int, P, P, P]
        L.oracle_hash_keys.restype = None
        L.oracle_hash_keys.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, P]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def fold_color(color_im: np.ndarray) -> np.ndarray:
    """grid_fusion.py:228-232: RGB (H,W,3) -> float32 B*65536 + G*256 + R."""
    c = color_im.astype(np.float32)
    return np.ascontiguousarray(np.floor(c[..., 2] * 65536 + c[..., 1] * 256 + c[..., 0]))


def volume_geometry(vol_bnds, voxel_size):
    """grid_fusion.py:31-44: dims = ceil(extent/vs) as int, origin = f32(min).
    Rewrites vol_bnds[:,1] in place exactly like the reference (when given an ndarray)."""
    vol_bnds = np.asarray(vol_bnds)
    assert vol_bnds.shape == (3, 2), "[!] `vol_bnds` should be of shape (3, 2)."
    vs = float(voxel_size)
    dims = np.ceil((vol_bnds[:, 1] - vol_bnds[:, 0]) / vs).copy(order="C").astype(int)
    vol_bnds[:, 1] = vol_bnds[:, 0] + dims * vs
    origin = vol_bnds[:, 0].copy(order="C").astype(np.float32)
    return vol_bnds, dims.astype(np.int64), origin, vs


class OracleTSDFVolume:
    """CPU oracle with TSDFVolume's semantics (grid_fusion.py:19-320, CPU mode).  `slab` =
    (x0, x1) keeps only that x-range of the volume; `x_index` keeps the listed global x rows
    (cyclic column shards).  Both are the multi-GPU partitions of DESIGN.md §6."""

    def __init__(self, vol_bnds, voxel_size, slab=None, x_index=None):
        self._vol_bnds, self._vol_dim, self._vol_origin, self._voxel_size = volume_geometry(
            vol_bnds, voxel_size)
        self._trunc_margin = 5 * self._voxel_size
        x0, x1 = (0, int(self._vol_dim[0])) if slab is None else slab
        self._off = np.array([x0, 0, 0], np.int64)
        self._xmap = None
        nxl = x1 - x0
        if x_index is not None:
            self._xmap = np.ascontiguousarray(x_index, dtype=np.int64)
            nxl = len(self._xmap)
        self._local_dim = np.array([nxl, self._vol_dim[1], self._vol_dim[2]], np.int64)
        shape = tuple(int(d) for d in self._local_dim)
        self._tsdf_vol_cpu = np.ones(shape, np.float32)
        self._weight_vol_cpu = np.zeros(shape, np.float32)
        self._color_vol_cpu = np.zeros(shape, np.float32)
        self.last_updated = None

    def integrate(self, color_im, depth_im, cam_intr, cam_pose, obs_weight=1.0, want_mask=False):
        im_h, im_w = depth_im.shape
        col = fold_color(color_im)
        depth = np.ascontiguousarray(depth_im, dtype=np.float64)
        K = np.ascontiguousarray(cam_intr, dtype=np.float64).reshape(9)
        Tinv = np.ascontiguousarray(np.linalg.inv(cam_pose), dtype=np.float64).reshape(16)
        upd = np.zeros(self._tsdf_vol_cpu.size, np.uint8) if want_mask else None
        n = lib().oracle_dense_integrate_rows(
            _p(self._local_dim), _p(self._off), _p(self._xmap), _p(self._vol_origin), self._voxel_size, self._trunc_margin,
            _p(self._tsdf_vol_cpu), _p(self._weight_vol_cpu), _p(self._color_vol_cpu),
            _p(depth), _p(col), im_h, im_w, _p(K), _p(Tinv), float(obs_weight), _p(upd))
        self.last_updated = upd
        return int(n)

    def get_volume(self):
        return self._tsdf_vol_cpu, self._color_vol_cpu


class OracleHashVolume:
    """CPU oracle with HashTable.integrate's per-voxel semantics (hash_fusion.py:103-145,
    voxel.py:19-49): float64 Voxel state, obs_weight ignored.  Dense-indexed storage."""

    def __init__(self, vol_bounds, voxel_size):
        self._vol_bounds, self._vol_dim, self._vol_origin, self._voxel_size = volume_geometry(
            vol_bounds, voxel_size)
        self._trunc_margin = 5 * self._voxel_size
        shape = tuple(int(d) for d in self._vol_dim)
        self.sdf = np.ones(shape, np.float64)
        self.weight = np.zeros(shape, np.float64)
        self.color = np.zeros(shape, np.float64)
        self.new_keys = None

    def integrate(self, color_im, depth_im, cam_intr, cam_pose, obs_weight=1.0):
        im_h, im_w = depth_im.shape
        col = fold_color(color_im)
        depth = np.ascontiguousarray(depth_im, dtype=np.float64)
        K = np.ascontiguousarray(cam_intr, dtype=np.float64).reshape(9)
        Tinv = np.ascontiguousarray(np.linalg.inv(cam_pose), dtype=np.float64).reshape(16)
        nk = np.zeros(self.sdf.size, np.uint8)
        n = lib().oracle_hash_integrate(
            _p(self._vol_dim), _p(self._vol_origin), self._voxel_size, self._trunc_margin,
            _p(self.sdf), _p(self.weight), _p(self.color), _p(depth), _p(col), im_h, im_w,
            _p(K), _p(Tinv), None, _p(nk))
        self.new_keys = np.flatnonzero(nk)  # C-order == reference insertion order
        return int(n)

    def entries(self):
        """(idx linear int64, sdf f64, weight f64, colour f64) of every voxel with an entry."""
        idx = np.flatnonzero(self.weight.reshape(-1) > 0)
        return (idx, self.sdf.reshape(-1)[idx], self.weight.reshape(-1)[idx],
                self.color.reshape(-1)[idx])


def hash_keys(xyz, table_size: int, int_bits: int = 64) -> np.ndarray:
    """hash_function (hash_fusion.py:182-190) for an (n,3) array of integer coordinates."""
    a = np.ascontiguousarray(np.asarray(xyz, dtype=np.int64).reshape(-1, 3))
    out = np.empty(a.shape[0], np.int64)
    lib().oracle_hash_keys(_p(a), a.shape[0], int(table_size), int(int_bits), _p(out))
    return out


# --------------------------------------------------------------------------------------------
# NumPy port (bench.py's timed CPU baseline, pinned by tests/test_oracle_golden.py against the
# reference-generated fixtures).  Same structure and arithmetic as the reference CPU path;
# numba-typed helpers restated as vectorised NumPy with the casts numba would emit.
# --------------------------------------------------------------------------------------------

def _numpy_project(vol, vox_coords, depth_im, cam_intr, cam_pose):
    """grid_fusion.py:260-290 (hash_fusion.py:113-131): valid voxels, their distance and pixel."""
    im_h, im_w = depth_im.shape
    # vox2world (:170-181): f64 multiply-add, rounded once to f32
    o = vol._vol_origin.astype(np.float64)
    cam_pts = (o[None, :] + vol._voxel_size * vox_coords.astype(np.float32).astype(np.float64)
               ).astype(np.float32)
    # rigid_transform (:363-368) with the reference's own np.dot
    xyz_h = np.hstack([cam_pts, np.ones((len(cam_pts), 1), dtype=np.float32)])
    cam_pts = np.dot(np.linalg.inv(cam_pose), xyz_h.T).T[:, :3]
    pix_z = cam_pts[:, 2]
    # cam2pix (:183-197)
    intr = cam_intr.astype(np.float32).astype(np.float64)
    with np.errstate(all="ignore"):
        pix_x = np.rint((cam_pts[:, 0] * intr[0, 0]) / pix_z + intr[0, 2]).astype(np.int64)
        pix_y = np.rint((cam_pts[:, 1] * intr[1, 1]) / pix_z + intr[1, 2]).astype(np.int64)
    valid_pix = (pix_x >= 0) & (pix_x < im_w) & (pix_y >= 0) & (pix_y < im_h) & (pix_z > 0)
    depth_val = np.zeros(pix_x.shape)
    depth_val[valid_pix] = depth_im[pix_y[valid_pix], pix_x[valid_pix]]
    depth_diff = depth_val - pix_z
    valid_pts = (depth_val > 0) & (depth_diff >= -vol._trunc_margin)
    dist = np.minimum(1, depth_diff / vol._trunc_margin)
    return valid_pts, dist[valid_pts], pix_x[valid_pts], pix_y[valid_pts]


def numpy_port_integrate(vol: OracleTSDFVolume, vox_coords, color_im, depth_im, cam_intr,
                         cam_pose, obs_weight=1.0):
    """grid_fusion.py:225-314 restated; `vox_coords` is the (N,3) int meshgrid of :158-168."""
    color = fold_color(color_im)
    valid_pts, valid_dist, px, py = _numpy_project(vol, vox_coords, depth_im, cam_intr, cam_pose)
    vx, vy, vz = (vox_coords[valid_pts, k] for k in range(3))
    w_old = vol._weight_vol_cpu[vx, vy, vz]
    tsdf_vals = vol._tsdf_vol_cpu[vx, vy, vz]
    # integrate_tsdf (:199-212) with numba's types
    w_new = (w_old.astype(np.float64) + obs_weight).astype(np.float32)
    t_new = (((w_old * tsdf_vals).astype(np.float64) + obs_weight * valid_dist)
             / w_new.astype(np.float64)).astype(np.float32)
    vol._weight_vol_cpu[vx, vy, vz] = w_new
    vol._tsdf_vol_cpu[vx, vy, vz] = t_new
    # colour (:302-314), float32 with NumPy 2 weak scalars
    old_color = vol._color_vol_cpu[vx, vy, vz]
    old_b = np.floor(old_color / 65536)
    old_g = np.floor((old_color - old_b * 65536) / 256)
    old_r = old_color - old_b * 65536 - old_g * 256
    new_color = color[py, px]
    new_b = np.floor(new_color / 65536)
    new_g = np.floor((new_color - new_b * 65536) / 256)
    new_r = new_color - new_b * 65536 - new_g * 256
    new_b = np.minimum(255., np.round((w_old * old_b + obs_weight * new_b) / w_new))
    new_g = np.minimum(255., np.round((w_old * old_g + obs_weight * new_g) / w_new))
    new_r = np.minimum(255., np.round((w_old * old_r + obs_weight * new_r) / w_new))
    vol._color_vol_cpu[vx, vy, vz] = new_b * 65536 + new_g * 256 + new_r
    return int(valid_pts.sum())


class NumpyPortHash:
    """HashTable's CPU integrate restated (hash_fusion.py:103-145): the vectorised projection,
    then the reference's per-voxel Python loop -- get_hash_entry, and on a miss a new Voxel,
    Voxel.integrate (data_structures/voxel.py:19-49, float64 state, np.round / np.minimum per
    voxel) and add_hash_entry -- over the chained-bucket table of bucket_table.BucketTable.
    obs_weight is not forwarded, as in the reference."""

    def __init__(self, vol_bounds, voxel_size, map_size=1000000, int_bits=64):
        from bucket_table import BucketTable
        self._vol_bounds, self._vol_dim, self._vol_origin, self._voxel_size = volume_geometry(
            vol_bounds, voxel_size)
        self._trunc_margin = 5 * self._voxel_size
        self.table = BucketTable(map_size, int_bits)
        self.sdf, self.weight, self.color = [], [], []  # per entry id (Voxel state)

    def _voxel_integrate(self, e, new_dist, new_color, obs_weight=1.0):
        w_old, d_old, c_old = self.weight[e], self.sdf[e], self.color[e]
        w_new = w_old + obs_weight
        self.sdf[e] = (d_old * w_old + new_dist * obs_weight) / w_new
        self.weight[e] = w_new
        old_b = np.floor(c_old / 65536)
        old_g = np.floor((c_old - old_b * 65536) / 256)
        old_r = c_old - old_b * 65536 - old_g * 256
        new_b = np.floor(new_color / 65536)
        new_g = np.floor((new_color - new_b * 65536) / 256)
        new_r = new_color - new_b * 65536 - new_g * 256
        bgr = np.minimum(255., np.round([(w_old * old_b + obs_weight * new_b) / w_new,
                                         (w_old * old_g + obs_weight * new_g) / w_new,
                                         (w_old * old_r + obs_weight * new_r) / w_new]))
        self.color[e] = bgr[0] * 65536 + bgr[1] * 256 + bgr[2]

    def integrate(self, vox_coords, color_im, depth_im, cam_intr, cam_pose, limit=None):
        """One frame; `limit` stops after that many valid voxels (a bounded timing sample).
        Returns the number of voxels integrated."""
        color = fold_color(color_im)
        valid_pts, valid_dist, px, py = _numpy_project(self, vox_coords, depth_im, cam_intr, cam_pose)
        coords = vox_coords[valid_pts]
        n = len(coords) if limit is None else min(limit, len(coords))
        t = self.table
        for i in range(n):
            pos = coords[i]
            e = t.get(pos)
            if e is None:
                e = len(t.pos)
                self.sdf.append(1.0)
                self.weight.append(0.0)
                self.color.append(0.0)
                self._voxel_integrate(e, valid_dist[i], color[py[i], px[i]])
                t.add(pos)
            else:
                self._voxel_integrate(e, valid_dist[i], color[py[i], px[i]])
        return n


def vox_coords_for(dims) -> np.ndarray:
    """grid_fusion.py:158-168 (meshgrid ij, (N,3) int)."""
    xv, yv, zv = np.meshgrid(range(int(dims[0])), range(int(dims[1])), range(int(dims[2])),
                             indexing="ij")
    return np.concatenate([xv.reshape(1, -1), yv.reshape(1, -1), zv.reshape(1, -1)],
                          axis=0).astype(int).T


def lounge_frame(i: int = 0):
    """Lounge frame i from the committed fixture copy (tests/golden/lounge), ingested like
    grid_demo1.py:80-84: depth u16 / 1000 with 65.535 -> 0, RGB, pose, intrinsics."""
    from PIL import Image
    root = os.path.join(os.path.dirname(_HERE), "tests", "golden", "lounge")
    d = np.array(Image.open(os.path.join(root, "frame-%06d.depth.png" % i))).astype(float) / 1000.0
    d[d == 65.535] = 0
    rgb = np.array(Image.open(os.path.join(root, "frame-%06d.color.jpg" % i)).convert("RGB"))
    pose = np.loadtxt(os.path.join(root, "frame-%06d.pose.txt" % i))
    K = np.loadtxt(os.path.join(root, "camera-intrinsics.txt"), delimiter=" ")
    return d, rgb, pose, K


def view_frustum(max_depth: float, H: int, W: int, K, pose) -> np.ndarray:
    """grid_fusion.py:371-383 for a frame whose max depth is `max_depth` (metres): (3, 5)."""
    out = np.zeros((3, 5))
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
    pose = np.ascontiguousarray(pose, dtype=np.float64).reshape(16)
    lib().oracle_view_frustum(float(max_depth), int(H), int(W), _p(K), _p(pose), _p(out))
    return out


def frustum_bounds(max_depths, H, W, K, poses, init=None) -> np.ndarray:
    """grid_demo1.py:50-64: running min/max of the frustum points, starting from `init`
    (the demo starts from zeros).  Returns (3, 2)."""
    b = np.zeros((3, 2)) if init is None else np.array(init, dtype=np.float64)
    for d, p in zip(max_depths, poses):
        v = view_frustum(d, H, W, K, p)
        b[:, 0] = np.minimum(b[:, 0], v.min(axis=1))
        b[:, 1] = np.maximum(b[:, 1], v.max(axis=1))
    return b
