#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container, where /root/reference (DiWu9/Union-Thesis-SLAM, read-only)
is mounted; it is a no-op elsewhere.  The reference is imported in a child process with
  PYTHONPATH = tools/refstubs : /root/reference     (numba/skimage are absent here)
  PYTHONDONTWRITEBYTECODE = 1                        (the reference tree is read-only)
and the numba-compiled helpers are replaced by NumPy versions with numba's typing
(`faithful_patch`), because an identity-`njit` stub would run vox2world in float32 under NumPy 2
weak-scalar rules and flip pixels.  rigid_transform (np.dot -> OpenBLAS dgemm)
and every other line of integrate() run as the reference wrote them.

Fixtures written (data only -- inputs and expected outputs, no reference source):
  golden/hash_kat.npz          hash_function KATs, int64 and int32-wrapping modes (G1)
  golden/lounge/               lounge frames 0-9 depth PNG, 0-2 colour JPG, poses, intrinsics
  golden/dense_c1.npz          lounge f0-f2 -> 128^3 @ 4 cm, reference grid CPU path, per frame (G2)
  golden/dense_c1_ow.npz       same with obs_weight = 1.0, 0.7, 2.5 (mixed f32/f64 colour path)
  golden/hash_c1.npz           lounge f0-f2 -> 128^3 @ 4 cm, reference HashTable.integrate (G2h)
  golden/synth_c1.npz          two synthetic frames (tsdf_amd.scene) -> 128^3 @ 8 cm room (G2s)
  golden/lounge2cm_kat.json    lounge 2 cm, frames 0-9: per-frame counts + final-state digest (G3)
  golden/lounge512_kat.json    lounge f0 -> 512^3 @ 2 cm: count + digest (G5)
  golden/frustum_bounds.npz    lounge frames 0-999: per-frame max depth (mm, after the demo's
                               65535 -> 0 masking), poses, and the reference get_view_frustum
                               points + the demo's running min/max bounds (G6)
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden")

LOUNGE_BNDS = [[-4.22106438, 3.86798203], [-2.6663104, 2.60146141], [0., 5.76272371]]
C1_BNDS = [[-2.56, 2.56], [-2.56, 2.56], [0.0, 5.12]]
C5_BNDS = [[-5.12, 5.12], [-5.12, 5.12], [-2.0, 8.24]]


def faithful_patch(grid_fusion, hash_fusion):
    """Numba-typing-faithful replacements for the @njit helpers (grid_fusion.py:170-212,
    hash_fusion.py:71-101)."""

    def vox2world(vol_origin, vox_coords, vox_size):
        o = vol_origin.astype(np.float32).astype(np.float64)
        c = vox_coords.astype(np.float32).astype(np.float64)
        return (o[None, :] + float(vox_size) * c).astype(np.float32)

    def cam2pix(cam_pts, intr):
        intr = intr.astype(np.float32).astype(np.float64)
        fx, fy, cx, cy = intr[0, 0], intr[1, 1], intr[0, 2], intr[1, 2]
        pix = np.empty((cam_pts.shape[0], 2), dtype=np.int64)
        with np.errstate(all="ignore"):
            pix[:, 0] = np.rint((cam_pts[:, 0] * fx) / cam_pts[:, 2] + cx).astype(np.int64)
            pix[:, 1] = np.rint((cam_pts[:, 1] * fy) / cam_pts[:, 2] + cy).astype(np.int64)
        return pix

    def integrate_tsdf(tsdf_vol, dist, w_old, obs_weight):
        w_new = (w_old.astype(np.float64) + float(obs_weight)).astype(np.float32)
        prod = (w_old.astype(np.float32) * tsdf_vol.astype(np.float32)).astype(np.float64)
        t = ((prod + float(obs_weight) * dist) / w_new.astype(np.float64)).astype(np.float32)
        return t, w_new

    grid_fusion.TSDFVolume.vox2world = staticmethod(vox2world)
    grid_fusion.TSDFVolume.cam2pix = staticmethod(cam2pix)
    grid_fusion.TSDFVolume.integrate_tsdf = staticmethod(integrate_tsdf)
    hash_fusion.HashTable.vox2world = staticmethod(vox2world)
    hash_fusion.HashTable.cam2pix = staticmethod(cam2pix)


def load_lounge(i, color=True):
    from PIL import Image
    d = np.array(Image.open(os.path.join(REF, "data", "frame-%06d.depth.png" % i)))
    depth = d.astype(float) / 1000.0
    depth[depth == 65.535] = 0
    pose = np.loadtxt(os.path.join(REF, "data", "frame-%06d.pose.txt" % i))
    rgb = None
    if color:
        rgb = np.array(Image.open(os.path.join(REF, "data", "frame-%06d.color.jpg" % i)).convert("RGB"))
    return d, depth, rgb, pose


def sparse_state(tsdf_obj):
    w = tsdf_obj._weight_vol_cpu.reshape(-1)
    idx = np.flatnonzero(w > 0).astype(np.int64)
    return (idx, tsdf_obj._tsdf_vol_cpu.reshape(-1)[idx].copy(), w[idx].copy(),
            tsdf_obj._color_vol_cpu.reshape(-1)[idx].copy())


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def inner():
    os.makedirs(GOLD, exist_ok=True)
    import grid_fusion  # noqa: E402  (the reference, via PYTHONPATH)
    import hash_fusion  # noqa: E402
    faithful_patch(grid_fusion, hash_fusion)
    cam_intr = np.loadtxt(os.path.join(REF, "data", "camera-intrinsics.txt"), delimiter=" ")
    only = set(sys.argv[sys.argv.index("--inner") + 1:])

    def want(name):
        return not only or name in only

    # ---- lounge inputs (data files copied as-is) --------------------------------------
    if want("lounge"):
        ld = os.path.join(GOLD, "lounge")
        os.makedirs(ld, exist_ok=True)
        shutil.copy(os.path.join(REF, "data", "camera-intrinsics.txt"), ld)
        shas = {}
        for i in range(10):
            for ext in ["depth.png", "pose.txt"] + (["color.jpg"] if i < 3 else []):
                shutil.copy(os.path.join(REF, "data", "frame-%06d.%s" % (i, ext)), ld)
            d, _, rgb, _ = load_lounge(i, color=i < 3)
            shas["frame-%06d.depth" % i] = digest(d)
            if rgb is not None:
                shas["frame-%06d.color" % i] = digest(rgb)
        with open(os.path.join(ld, "decoded_sha256.json"), "w") as f:
            json.dump(shas, f, indent=1, sort_keys=True)
        print("lounge inputs copied")

    # ---- G1 hash KATs ------------------------------------------------------------------
    if want("hash"):
        ht = hash_fusion.HashTable([[0, 0.04], [0, 0.04], [0, 0.04]], 0.02, 10, False)
        rng = np.random.default_rng(1234)
        coords = rng.integers(-1024, 1025, size=(256, 3)).astype(np.int64)
        coords = np.concatenate([coords, np.array([[80, 56, 0], [333, 234, 241], [342, 234, 241],
                                                   [332, 234, 242], [0, 0, 0], [-1, -1, -1]])])
        sizes = np.array([10, 1000, 100000, 1000000, 1 << 22], np.int64)
        out64 = np.empty((len(sizes), len(coords)), np.int64)
        out32 = np.empty_like(out64)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for si, n in enumerate(sizes):
                ht._table_size = int(n)
                for ci, c in enumerate(coords):
                    out64[si, ci] = int(ht.hash_function([np.int64(v) for v in c]))
                    out32[si, ci] = int(ht.hash_function([np.int32(v) for v in c]))
        np.savez_compressed(os.path.join(GOLD, "hash_kat.npz"), coords=coords, sizes=sizes,
                            h64=out64, h32=out32)
        print("hash KAT:", out64[2, -6:-2], out32[2, -6:-2])

    # ---- G2 dense config 1 -------------------------------------------------------------
    for name, ows in (("dense_c1", (1.0, 1.0, 1.0)), ("dense_c1_ow", (1.0, 0.7, 2.5))):
        if not want(name):
            continue
        vol = grid_fusion.TSDFVolume(np.array(C1_BNDS), 0.04, use_gpu=False)
        res = {"dims": np.asarray(vol._vol_dim), "origin": vol._vol_origin,
               "bounds_after": vol._vol_bnds, "obs_weight": np.array(ows)}
        prev = np.zeros(vol._weight_vol_cpu.shape, np.float32)
        for f in range(3):
            _, depth, rgb, pose = load_lounge(f)
            vol.integrate(rgb, depth, cam_intr, pose, obs_weight=ows[f])
            idx, t, w, c = sparse_state(vol)
            res["f%d_idx" % f], res["f%d_tsdf" % f], res["f%d_weight" % f], res["f%d_color" % f] = idx, t, w, c
            res["f%d_nupd" % f] = np.int64((vol._weight_vol_cpu != prev).sum())
            prev = vol._weight_vol_cpu.copy()
            print(name, "frame", f, "updated", int(res["f%d_nupd" % f]), "entries", len(idx),
                  "tsdf<1", int((t < 1).sum()))
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **res)

    # ---- G2h hash config 1 (reference per-voxel loop, ~2 s/frame) ------------------------
    if want("hash_c1"):
        ht = hash_fusion.HashTable(np.array(C1_BNDS), 0.04, 1000000, 0.75, False)
        res = {}
        for f in range(3):
            _, depth, rgb, pose = load_lounge(f)
            ht.integrate(rgb, depth, cam_intr, pose, obs_weight=1.0)
            pos, sdf, w, col = [], [], [], []
            for b in ht._hash_table:
                if b is None:
                    continue
                for j in range(5):
                    e = b.get_ith_entry(j)
                    if e is not None and e.get_voxel() is not None:
                        v = e.get_voxel()
                        pos.append([int(p) for p in e.get_position()])
                        sdf.append(float(v.get_sdf()))
                        w.append(float(v._weight))
                        col.append(float(v.get_color()))
            pos = np.array(pos, np.int64)
            order = np.lexsort((pos[:, 2], pos[:, 1], pos[:, 0]))
            res["f%d_pos" % f] = pos[order]
            res["f%d_sdf" % f] = np.array(sdf)[order]
            res["f%d_weight" % f] = np.array(w)[order]
            res["f%d_color" % f] = np.array(col)[order]
            res["f%d_entries" % f] = np.int64(ht.count_num_hash_entries())
            res["f%d_nonempty" % f] = np.int64(ht.get_num_non_empty_buckets())
            res["f%d_collisions" % f] = np.int64(ht.get_num_collisions())
            print("hash_c1 frame", f, "entries", len(pos), "buckets", ht.get_num_non_empty_buckets())
        np.savez_compressed(os.path.join(GOLD, "hash_c1.npz"), **res)

    # ---- G2s synthetic frames into 128^3 @ 8 cm of the room ----------------------------
    if want("synth"):
        sys.path.insert(0, os.path.join(REPO, "union-thesis-slam_amd"))
        from tsdf_amd import scene
        sp = scene.make_spheres(0)
        poses = scene.trajectory(1000, seed=0)[[0, 137]]
        depth_u16, rgb = scene.render(poses, sp, seed=0, start=0)
        depth_u16, rgb = depth_u16.numpy(), rgb.numpy()
        vol = grid_fusion.TSDFVolume(np.array([[0.0, 10.24]] * 3), 0.08, use_gpu=False)
        res = {"depth_u16": depth_u16, "rgb": rgb, "poses": poses, "K": scene.intrinsics()}
        prev = np.zeros(vol._weight_vol_cpu.shape, np.float32)
        for f in range(2):
            vol.integrate(rgb[f], scene.depth_metres(depth_u16[f]), scene.intrinsics(), poses[f])
            idx, t, w, c = sparse_state(vol)
            res["f%d_idx" % f], res["f%d_tsdf" % f], res["f%d_weight" % f], res["f%d_color" % f] = idx, t, w, c
            res["f%d_nupd" % f] = np.int64((vol._weight_vol_cpu != prev).sum())
            prev = vol._weight_vol_cpu.copy()
            print("synth frame", f, "updated", int(res["f%d_nupd" % f]))
        np.savez_compressed(os.path.join(GOLD, "synth_c1.npz"), **res)

    # ---- G3 lounge 2 cm, 10 frames -----------------------------------------------------
    if want("lounge2cm"):
        vol = grid_fusion.TSDFVolume(np.array(LOUNGE_BNDS), 0.02, use_gpu=False)
        kat = {"bounds": LOUNGE_BNDS, "voxel_size": 0.02, "dims": [int(d) for d in vol._vol_dim],
               "frames": []}
        prev = np.zeros(vol._weight_vol_cpu.shape, np.float32)
        for f in range(10):
            _, depth, rgb, pose = load_lounge(f, color=False)
            rgb = np.zeros(depth.shape + (3,), np.uint8)  # colour does not affect the voxel set
            vol.integrate(rgb, depth, cam_intr, pose)
            w = vol._weight_vol_cpu
            nupd = int((w != prev).sum())
            newk = int(((w > 0) & (prev == 0)).sum())
            prev = w.copy()
            kat["frames"].append({"updated": nupd, "new_keys": newk,
                                  "sum_weight": float(w.sum(dtype=np.float64))})
            print("lounge2cm frame", f, nupd, newk)
        idx, t, w, _ = sparse_state(vol)
        kat["unique"] = int(len(idx))
        kat["digest_idx_tsdf_weight"] = digest(idx, t, w)
        with open(os.path.join(GOLD, "lounge2cm_kat.json"), "w") as fh:
            json.dump(kat, fh, indent=1)

    # ---- G6 frustum bounds over the 1000 lounge frames -----------------------------------
    if want("frustum"):
        gen_frustum(grid_fusion, cam_intr)

    # ---- G5 lounge f0 -> 512^3 @ 2 cm --------------------------------------------------
    if want("lounge512"):
        vol = grid_fusion.TSDFVolume(np.array(C5_BNDS), 0.02, use_gpu=False)
        _, depth, rgb, pose = load_lounge(0)
        vol.integrate(rgb, depth, cam_intr, pose)
        idx, t, w, c = sparse_state(vol)
        kat = {"bounds": C5_BNDS, "voxel_size": 0.02, "dims": [int(d) for d in vol._vol_dim],
               "updated": int(len(idx)), "digest_idx_tsdf_weight_color": digest(idx, t, w, c)}
        print("lounge512", kat)
        with open(os.path.join(GOLD, "lounge512_kat.json"), "w") as fh:
            json.dump(kat, fh, indent=1)


def gen_frustum(grid_fusion, cam_intr):
    """G6: grid_demo1.py:50-64 over the 1000 lounge frames.  get_view_frustum only reads the
    image shape and np.max(depth), so it is called on a zero image of the frame's shape holding
    the frame's max depth at one pixel -- exactly the reference computation, without shipping
    1000 depth images."""
    from PIL import Image
    n = 1000
    max_mm = np.zeros(n, np.uint16)
    poses = np.zeros((n, 4, 4))
    pts = np.zeros((n, 3, 5))
    bnds_run = np.zeros((n, 3, 2))
    vol_bnds = np.zeros((3, 2))
    for i in range(n):
        d = np.array(Image.open(os.path.join(REF, "data", "frame-%06d.depth.png" % i)))
        depth_im = d.astype(float) / 1000.0
        depth_im[depth_im == 65.535] = 0
        m = int(np.max(np.where(d == 65535, 0, d)))
        assert np.max(depth_im) == m / 1000.0
        max_mm[i] = m
        poses[i] = np.loadtxt(os.path.join(REF, "data", "frame-%06d.pose.txt" % i))
        proxy = np.zeros(d.shape)
        proxy[0, 0] = m / 1000.0
        vfp = grid_fusion.get_view_frustum(proxy, cam_intr, poses[i])
        pts[i] = vfp
        vol_bnds[:, 0] = np.minimum(vol_bnds[:, 0], np.amin(vfp, axis=1))
        vol_bnds[:, 1] = np.maximum(vol_bnds[:, 1], np.amax(vfp, axis=1))
        bnds_run[i] = vol_bnds
    np.savez_compressed(os.path.join(GOLD, "frustum_bounds.npz"), max_depth_mm=max_mm, poses=poses,
                        intr=cam_intr, shape=np.array(d.shape), frustum_pts=pts, bounds_running=bnds_run,
                        bounds=vol_bnds)
    print("frustum bounds", vol_bnds.tolist())


def main():
    if not os.path.isdir(REF):
        print("gen_golden: /root/reference absent; nothing to do")
        return
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(REPO, "tools", "refstubs"), REF])
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    env.setdefault("OPENBLAS_NUM_THREADS", "8")
    cmd = [sys.executable, os.path.abspath(__file__), "--inner"] + sys.argv[1:]
    sys.exit(subprocess.run(cmd, env=env, cwd="/tmp").returncode)


if __name__ == "__main__":
    if "--inner" in sys.argv:
        inner()
    else:
        main()
