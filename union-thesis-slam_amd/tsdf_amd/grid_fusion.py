"""Dense TSDF volume on MI355X -- drop-in for `grid_fusion.TSDFVolume` (grid_fusion.py:19-320).

Same constructor, same `integrate()` / `get_volume()` signatures and results as the
reference's CPU path (bit-exact voxel set, tsdf, weight and colour; tests/test_dense_gpu.py).
The work runs in hand-written gfx950 kernels behind the C-ABI of include/tsdf_hip.h; this
module only does the reference's host-side duties:

  * volume geometry, including the in-place rewrite of vol_bnds[:,1] (grid_fusion.py:31-44);
  * inv(cam_pose) with NumPy/LAPACK, as the reference does on the host (grid_fusion.py:265);
  * the colour fold for non-uint8 input (grid_fusion.py:228-232);
  * depth: float64 metres are sent as they are (uint16 millimetres when the caller has them);
  * per-frame integrate() calls are deferred into pinned staging batches of 8 frames (TSDF_DEFER)
    that run as one temporally batched launch; every other call (get_volume, get_state, stats,
    sync, meshing, batch integrate) runs the pending frames first, so results and their order
    are those of one-by-one integration.  `defer=False` makes each call synchronous.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _ffi, sharding
from .ply import meshwrite, pcwrite  # noqa: F401  (grid_fusion.meshwrite / pcwrite, as in the reference)


def volume_geometry(vol_bnds, voxel_size):
    """grid_fusion.py:31-44: dims = ceil(extent/vs), vol_bnds[:,1] rewritten in place,
    origin = f32(vol_bnds[:,0])."""
    vol_bnds = np.asarray(vol_bnds)
    assert vol_bnds.shape == (3, 2), "[!] `vol_bnds` should be of shape (3, 2)."
    vs = float(voxel_size)
    dims = np.ceil((vol_bnds[:, 1] - vol_bnds[:, 0]) / vs).copy(order="C").astype(int)
    vol_bnds[:, 1] = vol_bnds[:, 0] + dims * vs
    origin = vol_bnds[:, 0].copy(order="C").astype(np.float32)
    return vol_bnds, dims, origin, vs


def encode_depth(depth_im):
    """(kind, contiguous array) for the C-ABI.  uint16 input is taken as millimetres; anything
    else goes as float64 metres, the reference's own depth_im, read by the kernels as is (no host
    pass over the image)."""
    d = np.asarray(depth_im)
    if d.dtype == np.uint16:
        return _ffi.DEPTH_U16_MM, np.ascontiguousarray(d)
    return _ffi.DEPTH_F64_M, np.ascontiguousarray(d, dtype=np.float64)


def encode_color(color_im):
    """uint8 RGB goes as is (the kernel folds it); anything else is folded here exactly like
    grid_fusion.py:228-232 and sent as float32."""
    c = np.asarray(color_im)
    if c.dtype == np.uint8 and c.ndim == 3 and c.shape[2] == 3:
        return _ffi.COLOR_RGB8, np.ascontiguousarray(c)
    c = c.astype(np.float32)
    folded = np.floor(c[..., 2] * (256 * 256) + c[..., 1] * 256 + c[..., 0])
    return _ffi.COLOR_F32, np.ascontiguousarray(folded, dtype=np.float32)


def frame_stack(depth, depth_kind, color, color_kind, device_ptrs):
    """Frame-stack kinds for the batch entry points: default u16 mm / RGB8 for device
    pointers; for host arrays, taken from (and checked against) the dtypes -- u16|i16 mm or
    f64 m depth (F,H,W); (F,H,W,3) u8 or folded (F,H,W) f32 colour."""
    if device_ptrs or isinstance(depth, int):  # raw addresses (device, or pinned host)
        return (depth, _ffi.DEPTH_U16_MM if depth_kind is None else depth_kind,
                color, _ffi.COLOR_RGB8 if color_kind is None else color_kind)
    depth, color = np.ascontiguousarray(depth), np.ascontiguousarray(color)
    dk = {np.dtype(np.uint16): _ffi.DEPTH_U16_MM, np.dtype(np.int16): _ffi.DEPTH_U16_MM,
          np.dtype(np.float64): _ffi.DEPTH_F64_M}.get(depth.dtype)
    ck = (_ffi.COLOR_RGB8 if color.dtype == np.uint8 and color.ndim == 4 else
          _ffi.COLOR_F32 if color.dtype == np.float32 and color.ndim == 3 else None)
    if dk is None or ck is None or depth.ndim != 3 or color.shape[:3] != depth.shape:
        raise ValueError(f"depth {depth.dtype}{depth.shape} / colour {color.dtype}{color.shape} "
                         "is not a supported frame stack")
    if (depth_kind is not None and depth_kind != dk) or (color_kind is not None and color_kind != ck):
        raise ValueError("depth_kind/color_kind disagree with the array dtypes")
    return depth, dk, color, ck


class TSDFVolume:
    """Volumetric TSDF Fusion of RGB-D Images, on an MI355X.

    Args (as grid_fusion.py:22-29):
      vol_bnds (ndarray): (3, 2) xyz bounds (min/max) in metres; column 1 is rewritten.
      voxel_size (float): metres.
      use_gpu: accepted for signature compatibility; the volume always lives in HBM.
    Extra keyword-only args (slab sharding):
      device: HIP device index.  slab: (x_begin, x_end) voxel range of this shard along x.
      shard: (rank, world) cyclic brick-column shard (sharding.columns) -- the bench's layout.
      `x_index` holds the global x of every local x row either way.
      defer: integrate() collects frames into batches of 8 (TSDF_DEFER); False: one synchronous
      call per frame.
    """

    def __init__(self, vol_bnds, voxel_size, use_gpu=True, *, device=0, slab=None, shard=None,
                 defer=True):
        print("Initializing voxel grids ... ")
        self.defer = bool(defer)
        self._vol_bnds, self._vol_dim, self._vol_origin, self._voxel_size = volume_geometry(
            vol_bnds, voxel_size)
        self._trunc_margin = 5 * self._voxel_size
        self._color_const = 256 * 256
        print("Voxel volume size: {} x {} x {} - # points: {:,}".format(
            self._vol_dim[0], self._vol_dim[1], self._vol_dim[2],
            self._vol_dim[0] * self._vol_dim[1] * self._vol_dim[2]))
        self.gpu_mode = True
        self.device = int(device)
        origin = np.ascontiguousarray(self._vol_origin, dtype=np.float32)
        h = ctypes.c_void_p()
        if shard is not None:
            if slab is not None:
                raise ValueError("give slab or shard, not both")
            rank, world = int(shard[0]), int(shard[1])
            self.x_index = sharding.columns(rank, world, int(self._vol_dim[0]))
            self.slab = None
            gdims = np.ascontiguousarray(self._vol_dim, dtype=np.int64)
            _ffi.call("tsdf_dense_create_shard", _ffi.ptr(gdims), rank, world, _ffi.ptr(origin),
                      self._voxel_size, float(self._trunc_margin), self.device, ctypes.byref(h))
        else:
            x0, x1 = (0, int(self._vol_dim[0])) if slab is None else (int(slab[0]), int(slab[1]))
            if not (0 <= x0 < x1 <= int(self._vol_dim[0])):
                raise ValueError(f"slab {slab} outside [0, {self._vol_dim[0]})")
            self.slab = (x0, x1)
            self.x_index = np.arange(x0, x1, dtype=np.int64)
            dims = np.array([x1 - x0, self._vol_dim[1], self._vol_dim[2]], np.int64)
            off = np.array([x0, 0, 0], np.int64)
            _ffi.call("tsdf_dense_create", _ffi.ptr(dims), _ffi.ptr(off), _ffi.ptr(origin),
                      self._voxel_size, float(self._trunc_margin), self.device, ctypes.byref(h))
        self._local_dim = np.array([len(self.x_index), self._vol_dim[1], self._vol_dim[2]], np.int64)
        self._h = h

    # ------------------------------------------------------------------ reference API
    def integrate(self, color_im, depth_im, cam_intr, cam_pose, obs_weight=1.):
        """Integrate an RGB-D frame (grid_fusion.py:214-314).

        color_im (H,W,3) RGB, depth_im (H,W) metres, cam_intr (3,3), cam_pose (4,4)
        camera-to-world, obs_weight float."""
        im_h, im_w = np.shape(depth_im)[:2]
        dk, d = encode_depth(depth_im)
        ck, c = encode_color(color_im)
        if c.shape[:2] != (im_h, im_w):
            raise ValueError("color_im and depth_im sizes differ")
        K = _ffi.f64(cam_intr, 9)
        Tinv = _ffi.f64(np.linalg.inv(np.asarray(cam_pose, dtype=np.float64)), 16)
        _ffi.call("tsdf_dense_integrate", self._h, _ffi.ptr(d), dk, _ffi.ptr(c), ck, im_h, im_w,
                  _ffi.ptr(K), _ffi.ptr(Tinv), float(obs_weight), _ffi.DEFER if self.defer else 0)

    def get_volume(self):
        """(tsdf, colour) float32 C-order (X,Y,Z) host arrays (grid_fusion.py:316-320)."""
        t, _, c = self.get_state(weight=False)
        return t, c

    # ------------------------------------------------------------------ extensions
    def get_state(self, weight=True):
        shape = tuple(int(x) for x in self._local_dim)
        t = np.empty(shape, np.float32)
        w = np.empty(shape, np.float32) if weight else None
        c = np.empty(shape, np.float32)
        _ffi.call("tsdf_dense_get", self._h, _ffi.ptr(t), _ffi.ptr(w), _ffi.ptr(c))
        return t, w, c

    def get_weight(self):
        return self.get_state(weight=True)[1]

    def set_state(self, tsdf, weight, color):
        a = [None if x is None else np.ascontiguousarray(x, dtype=np.float32) for x in (tsdf, weight, color)]
        _ffi.call("tsdf_dense_set", self._h, *[_ffi.ptr(x) for x in a])

    def integrate_batch(self, depth, color, cam_intr, world_to_cam, obs_weight=None, *,
                        depth_kind=None, color_kind=None, hw=None, device_ptrs=False, sync=True,
                        invalid_65535=False):
        """F frames back to back on the volume's stream (the bench's step).

        depth/color: host ndarrays (F,H,W[,3]) or, with device_ptrs=True, integer device
        addresses of such arrays already resident in HBM (then hw=(H,W) is required).
        world_to_cam: (F,4,4) = inv(cam_pose) per frame, computed by the caller.
        depth_kind/color_kind default to u16 mm / RGB8 for device pointers and are taken from
        the dtype of host arrays (u16|i16 mm or f64 m; (F,H,W,3) u8 or folded (F,H,W) f32).
        Host arrays are copied by host threads into page-locked bounce slots and DMAed into
        one of four device staging slots while earlier batches integrate.  invalid_65535: u16 65535 mm is invalid (0),
        the demos' `depth_im[depth_im == 65.535] = 0` (grid_demo1.py:82) done on the device."""
        depth, depth_kind, color, color_kind = frame_stack(depth, depth_kind, color, color_kind, device_ptrs)
        T = np.ascontiguousarray(np.asarray(world_to_cam, dtype=np.float64).reshape(-1, 16))
        n = T.shape[0]
        H, W = hw if (device_ptrs or isinstance(depth, int)) else np.shape(depth)[1:3]
        ow = None if obs_weight is None else _ffi.f64(obs_weight, n)
        flags = ((_ffi.DEVICE_PTRS if device_ptrs else 0) | (0 if sync else _ffi.ASYNC) |
                 (_ffi.DEPTH_INVALID_65535 if invalid_65535 else 0))
        _ffi.call("tsdf_dense_integrate_batch", self._h, n, _ffi.ptr(depth), depth_kind,
                  _ffi.ptr(color), color_kind, int(H), int(W), _ffi.ptr(_ffi.f64(cam_intr, 9)),
                  _ffi.ptr(T), _ffi.ptr(ow), flags)

    def sync(self):
        _ffi.call("tsdf_dense_sync", self._h)

    def frames_per_launch(self):
        """Frames one launch integrates (the temporal batch, tsdf_dense_frames_per_launch)."""
        if not hasattr(_ffi.load(), "tsdf_dense_frames_per_launch"):  # (an older build under A/B)
            return 8
        n = ctypes.c_int(0)
        _ffi.call("tsdf_dense_frames_per_launch", self._h, ctypes.byref(n))
        return n.value

    def stats(self, reset=False):
        s = _ffi.Stats()
        _ffi.call("tsdf_dense_stats", self._h, ctypes.byref(s), int(bool(reset)))
        return s.as_dict()

    def set_profiling(self, on=True):
        _ffi.call("tsdf_dense_set_profiling", self._h, int(bool(on)))

    def reset(self):
        _ffi.call("tsdf_dense_reset", self._h)

    def extract_mesh(self, normals=True, colors=True, faces=True, halo=None, global_x=None, keys=False):
        """Marching cubes at level 0 on the device (tsdf_dense_extract_mesh): (verts (N,3) f32
        world, normals (N,3) f32, colors (N,3) u8, faces (M,3) i32[, keys (N,) int64]); a field not
        asked for is None.  A shard of a multi-GPU volume passes its neighbours' border rows:
        halo = (global x (n,), tsdf (n,Y,Z), colour (n,Y,Z)) as numpy arrays or CUDA tensors
        (sharding.mesh_shard does the exchange), global_x = the unsharded x extent."""
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        if halo is None and global_x is None:
            _ffi.call("tsdf_dense_extract_mesh", self._h, ctypes.byref(nv), ctypes.byref(nt))
        else:
            gx, ht, hc = halo if halo is not None else (np.zeros(0, np.int64), None, None)
            gx = np.ascontiguousarray(np.asarray(gx, dtype=np.int64))
            dev = ht is not None and not isinstance(ht, np.ndarray)
            if dev:
                hp, cp = ht.data_ptr(), hc.data_ptr()
            else:
                ht = None if ht is None else np.ascontiguousarray(ht, dtype=np.float32)
                hc = None if hc is None else np.ascontiguousarray(hc, dtype=np.float32)
                hp, cp = _ffi.ptr(ht), _ffi.ptr(hc)
            _ffi.call("tsdf_dense_extract_mesh_halo", self._h, int(global_x or self._vol_dim[0]), _ffi.ptr(gx),
                      len(gx), hp, cp, _ffi.DEVICE_PTRS if dev else 0, ctypes.byref(nv), ctypes.byref(nt))
        v = np.empty((nv.value, 3), np.float32)
        n = np.empty((nv.value, 3), np.float32) if normals else None
        c = np.empty((nv.value, 3), np.uint8) if colors else None
        f = np.empty((nt.value, 3), np.int32) if faces else None
        _ffi.call("tsdf_dense_get_mesh", self._h, _ffi.ptr(v), _ffi.ptr(n), _ffi.ptr(c), _ffi.ptr(f))
        if not keys:
            return v, n, c, f
        k = np.empty(nv.value, np.int64)
        _ffi.call("tsdf_dense_get_mesh_keys", self._h, _ffi.ptr(k))
        return v, n, c, f, k

    def mesh_halo_rows(self, global_x=None):
        """Global x rows this shard's marching cubes reads but does not own (sorted)."""
        gx = int(global_x or self._vol_dim[0])
        n = ctypes.c_int64(0)
        _ffi.call("tsdf_dense_mesh_halo_rows", self._h, gx, None, ctypes.byref(n))
        rows = np.empty(n.value, np.int64)
        _ffi.call("tsdf_dense_mesh_halo_rows", self._h, gx, _ffi.ptr(rows), ctypes.byref(n))
        return rows

    def get_rows(self, local_rows, weight=True, out=None):
        """Local x rows in C-order (n, Y, Z): numpy (tsdf, weight, colour), or, with out = three
        CUDA tensors (or None entries), filled on the device (no host copy)."""
        rows = np.ascontiguousarray(np.asarray(local_rows, dtype=np.int64).reshape(-1))
        if out is not None:
            ptrs = [0 if o is None else o.data_ptr() for o in out]
            _ffi.call("tsdf_dense_get_rows", self._h, _ffi.ptr(rows), len(rows),
                      *[p if p else None for p in ptrs], _ffi.DEVICE_PTRS)
            return out
        shape = (len(rows), int(self._local_dim[1]), int(self._local_dim[2]))
        t, c = np.empty(shape, np.float32), np.empty(shape, np.float32)
        w = np.empty(shape, np.float32) if weight else None
        _ffi.call("tsdf_dense_get_rows", self._h, _ffi.ptr(rows), len(rows), _ffi.ptr(t), _ffi.ptr(w),
                  _ffi.ptr(c), 0)
        return t, w, c

    def get_point_cloud(self):
        """grid_fusion.py:322-338: (N, 6) float32 rows x, y, z, r, g, b of the mesh vertices."""
        v, _, c, _ = self.extract_mesh(normals=False, faces=False)
        return np.hstack([v, c])

    def get_mesh(self):
        """grid_fusion.py:340-360: (verts, faces, norms, colors) from marching cubes on the device."""
        v, n, c, f = self.extract_mesh()
        return v, f, n, c

    def close(self):
        if getattr(self, "_h", None):
            _ffi.call("tsdf_dense_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rigid_transform(xyz, transform):
    """grid_fusion.py:363-368 (host helper used by the demos' bounds estimation)."""
    xyz_h = np.hstack([xyz, np.ones((len(xyz), 1), dtype=np.float32)])
    xyz_t_h = np.dot(transform, xyz_h.T).T
    return xyz_t_h[:, :3]


def get_view_frustum(depth_im, cam_intr, cam_pose):
    """grid_fusion.py:371-383: the camera origin and the four image corners pushed out to the
    frame's max depth, in world coordinates, as a (3, 5) array."""
    h, w = depth_im.shape[:2]
    dmax = np.max(depth_im)
    z = np.array([0.0, dmax, dmax, dmax, dmax])
    u = np.array([0, 0, 0, w, w])
    v = np.array([0, 0, h, 0, h])
    cam = np.stack([(u - cam_intr[0, 2]) * z / cam_intr[0, 0],
                    (v - cam_intr[1, 2]) * z / cam_intr[1, 1], z], axis=1)
    return rigid_transform(cam, cam_pose).T


def view_frustum_bounds(depth_frames, cam_intr, cam_poses, init=None, *, invalid_65535=False,
                        device=0, device_ptrs=False, hw=None, depth_kind=None, n_frames=None,
                        return_max_depth=False, return_points=False):
    """Volume bounds from the union of the frames' view frustums, on the GPU: the demo loop
    grid_demo1.py:50-64 (hash_demo1.py:93-107) over get_view_frustum (grid_fusion.py:371-383).

    depth_frames: (F,H,W) u16 millimetres or f64 metres (host), or with device_ptrs=True a device
    address of F such frames (then hw=(H,W), n_frames=F and depth_kind are required).
    cam_poses: (F,4,4) camera-to-world.  init: starting (3,2) bounds; the demo starts from zeros.
    invalid_65535: u16 65535 mm counts as 0 (the demos' `depth_im[depth_im == 65.535] = 0`).
    Returns the (3,2) bounds [, per-frame max depth (F,)] [, frustum points (F,3,5)]."""
    poses = np.ascontiguousarray(np.asarray(cam_poses, dtype=np.float64).reshape(-1, 16))
    F = poses.shape[0]
    if device_ptrs:
        if hw is None or depth_kind is None or n_frames is None:
            raise ValueError("device_ptrs needs hw, depth_kind and n_frames")
        H, W = hw
        dk, d = depth_kind, depth_frames
        if n_frames != F:
            raise ValueError("n_frames differs from the number of poses")
    else:
        d = np.ascontiguousarray(depth_frames)
        if d.ndim != 3 or d.shape[0] != F:
            raise ValueError(f"depth_frames {d.shape} does not match {F} poses")
        dk = {np.dtype(np.uint16): _ffi.DEPTH_U16_MM, np.dtype(np.int16): _ffi.DEPTH_U16_MM,
              np.dtype(np.float64): _ffi.DEPTH_F64_M}.get(d.dtype)
        if dk is None:
            raise ValueError(f"depth dtype {d.dtype}: use uint16 millimetres or float64 metres")
        if depth_kind is not None and depth_kind != dk:
            raise ValueError("depth_kind disagrees with the array dtype")
        H, W = d.shape[1:]
    b = np.zeros((3, 2)) if init is None else np.array(init, dtype=np.float64).reshape(3, 2)
    b = np.ascontiguousarray(b)
    md = np.empty(F) if return_max_depth else None
    pts = np.empty((F, 3, 5)) if return_points else None
    flags = (_ffi.DEVICE_PTRS if device_ptrs else 0) | (_ffi.DEPTH_INVALID_65535 if invalid_65535 else 0)
    _ffi.call("tsdf_frustum_bounds", _ffi.ptr(d), dk, F, int(H), int(W), _ffi.ptr(_ffi.f64(cam_intr, 9)),
              _ffi.ptr(poses), flags, int(device), _ffi.ptr(md), _ffi.ptr(pts), _ffi.ptr(b))
    out = [b]
    if return_max_depth:
        out.append(md)
    if return_points:
        out.append(pts)
    return out[0] if len(out) == 1 else tuple(out)
