"""Where the time of a fused launch goes, hash against dense, on one GPU (diagnostic build:
tools/build_variant.sh wgt "-DTSDF_WG_TIMES", run with TSDF_HIP_LIB=abtest/libwgt.so).  The bench's
driver window (a fresh volume / table, 5 batches, then calls of 4 batches: the second launch of each
call runs all three stages) into a fresh dense volume, a fresh hash table (inserting) and the same hash
table again (every block exists).  Per role: workgroups, first / last start, median / last end,
mean busy time (us from the launch's first workgroup start).  One JSON line per configuration.

    PYTHONPATH=union-thesis-slam_amd TSDF_HIP_LIB=abtest/libwgt.so python tools/gpu/wg_times_hash.py
"""
import contextlib
import ctypes
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene  # noqa: E402

NW = 16384


def summarize(buf):
    t0 = buf[0].astype(np.int64)
    keep = buf[1] != 0  # (the library clears the buffer at each read: this call's launches only)
    t0 = t0[keep]
    t1 = buf[1][keep].astype(np.int64)
    role = (buf[2][keep] >> np.uint64(32)).astype(np.int64)
    it = (buf[2][keep] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0
    r = {"span": float(e.max())}
    for code, name in ((0, "integrate"), (1, "cull"), (2, "prep")):
        m = role == code
        if m.any():
            r[name] = [int(m.sum()), float(s[m].min()), float(s[m].max()), float(np.median(e[m])), float(e[m].max()),
                       float((e[m] - s[m]).mean())]
    r["items"] = float(it[role == 0].mean()) if (role == 0).any() else 0.0
    m = role == 0
    if m.any():  # the integrate workgroups by XCD (XCC_ID), and whether the last ones took more items
        xcc = (buf[3][keep] >> np.uint64(32)).astype(np.int64)
        r["xcd_end_median"] = [float(np.median(e[m & (xcc == x)])) if (m & (xcc == x)).any() else 0.0 for x in range(8)]
        r["xcd_end_max"] = [float(e[m & (xcc == x)].max()) if (m & (xcc == x)).any() else 0.0 for x in range(8)]
        late = m & (e >= np.quantile(e[m], 0.9))
        r["items_late_over_mean"] = float(it[late].mean() / max(1e-9, it[m].mean()))
        # the two integrate workgroups of a CU (XCC, SE/SH/CU bits of HW_ID): how far apart they end,
        # and how often the later-dispatched one (higher workgroup id) ends last
        hw = (buf[3][keep] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        wid = np.flatnonzero(keep)
        cu = xcc * 4096 + ((hw >> 8) & 0xFF)
        gaps, later_last = [], []
        for c in np.unique(cu[m]):
            sel = np.flatnonzero(m & (cu == c))
            if len(sel) == 2:
                a, b2 = sel[np.argsort(wid[sel])]
                gaps.append(abs(e[b2] - e[a]))
                later_last.append(e[b2] > e[a])
        r["cu_pair_gap_mean"] = float(np.mean(gaps)) if gaps else 0.0
        r["cu_pair_later_ends_last"] = float(np.mean(later_last)) if later_last else 0.0
        r["cu_pairs"] = len(gaps)
    return r


def main():
    dev = torch.device("cuda", 0)
    F = 800  # (25 batches of up to 32 frames)
    poses = scene.trajectory(F, seed=0, radius_frac=scene.BENCH_RING)
    sph = scene.make_spheres(0, ring_frac=scene.BENCH_RING)
    depth = torch.empty((F, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((F, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, F, 50):
        d, c = scene.render(poses[s:s + 50], sph, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    K = scene.intrinsics()
    bnds = np.array([[0.0, 10.24]] * 3)
    ds, cs = depth[0].numel() * 2, rgb[0].numel()
    lib = _ffi.load()
    fns = {"dense": lib.tsdf_diag_wg_times, "hash": lib.tsdf_diag_wg_times_hash}
    for fn in fns.values():
        fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros((4, NW), np.uint64)

    def run(kind, v, label):
        B = v.frames_per_launch()
        v.integrate_batch(depth.data_ptr(), rgb.data_ptr(), K, Tinv[:5 * B], hw=(480, 640), device_ptrs=True)
        rows = []
        for start in range(5 * B, 25 * B - 4 * B + 1, 4 * B):  # 4 batches a call: launch 1 runs all three stages
            v.integrate_batch(depth.data_ptr() + start * ds, rgb.data_ptr() + start * cs, K, Tinv[start:start + 4 * B],
                              hw=(480, 640), device_ptrs=True, sync=False)
            v.sync()
            fns[kind](buf.ctypes.data)
            rows.append(summarize(buf))
        out = {"config": label, "span_us": round(float(np.mean([r["span"] for r in rows])), 2),
               "items_mean": round(float(np.mean([r["items"] for r in rows])), 1)}
        if all("xcd_end_median" in r for r in rows):
            out["integrate_xcd_end_median_us"] = [round(float(x), 1) for x in np.mean([r["xcd_end_median"] for r in rows], axis=0)]
            out["integrate_xcd_end_max_us"] = [round(float(x), 1) for x in np.mean([r["xcd_end_max"] for r in rows], axis=0)]
            out["integrate_late10_items_over_mean"] = round(float(np.mean([r["items_late_over_mean"] for r in rows])), 3)
            out["integrate_cu_pair_gap_us"] = round(float(np.mean([r["cu_pair_gap_mean"] for r in rows])), 1)
            out["integrate_cu_pair_later_ends_last"] = round(float(np.mean([r["cu_pair_later_ends_last"] for r in rows])), 3)
            out["integrate_cu_pairs"] = int(np.mean([r["cu_pairs"] for r in rows]))
        for name in ("integrate", "cull", "prep"):
            vv = np.array([r[name] for r in rows if name in r])
            if len(vv):
                out[name] = {"wgs": int(vv[0, 0]), "first_start_us": round(float(vv[:, 1].mean()), 2),
                             "last_start_us": round(float(vv[:, 2].mean()), 2),
                             "end_median_us": round(float(vv[:, 3].mean()), 2),
                             "last_end_us": round(float(vv[:, 4].mean()), 2),
                             "busy_mean_us": round(float(vv[:, 5].mean()), 2)}
        print(json.dumps(out), flush=True)

    with contextlib.redirect_stdout(io.StringIO()):
        vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02)
    for rep in range(2):  # (the first pass warms the clocks)
        vol.reset()
        run("dense", vol, f"dense, driver window, pass {rep}")
    vol.close()
    with contextlib.redirect_stdout(io.StringIO()):
        ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, max_blocks=1 << 15)
    run("hash", ht, "hash, driver window, fresh table (inserting)")
    run("hash", ht, "hash, driver window again (every block exists)")
    ht.close()
    with contextlib.redirect_stdout(io.StringIO()):
        ht = hash_fusion.HashTable(bnds.copy(), 0.02, 1 << 22, shard=0, n_shards=8, max_blocks=1 << 15)
    run("hash", ht, "hash bucket-range shard 0 of 8, fresh (inserting)")
    run("hash", ht, "hash bucket-range shard 0 of 8 again (every block exists)")
    ht.close()


if __name__ == "__main__":
    main()
