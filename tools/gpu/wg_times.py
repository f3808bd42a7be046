"""Where the time of an eighth-shard launch goes: per workgroup of the last fused launch of a call
(integrate, cull and prep roles), its start, end, list items and the CU it ran on (diagnostic build: tools/build_variant.sh wgt
"-DTSDF_WG_TIMES", run with TSDF_HIP_LIB=abtest/libwgt.so).  Bench workload (scaling_sim's), one
GPU and rank 0 of 2 / 4 / 8 cyclic column shards.  Prints one JSON line per configuration."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "union-thesis-slam_amd"))
from tsdf_amd import _ffi, grid_fusion, scene  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    F = 400
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
    fn = lib.tsdf_diag_wg_times
    fn.argtypes = [ctypes.c_void_p]
    NW = 16384
    buf = np.zeros((4, NW), np.uint64)
    for world in (1, 2, 4, 8):
        vol = grid_fusion.TSDFVolume(bnds.copy(), 0.02, shard=(0, world))
        rows = []
        B = vol.frames_per_launch()
        for start in range(0, F - 4 * B + 1, 4 * B):  # 4 batches a call: its launch 1 runs all three stages
            vol.integrate_batch(depth.data_ptr() + start * ds, rgb.data_ptr() + start * cs, K,
                                Tinv[start:start + 4 * B], hw=(480, 640), device_ptrs=True)
            if start == 0:
                continue
            fn(buf.ctypes.data)
            t0 = buf[0].astype(np.int64)
            keep = buf[1] != 0  # (the library clears the buffer at each read: this call's launches only)
            t0 = t0[keep]
            t1 = buf[1][keep].astype(np.int64)
            role = (buf[2][keep] >> np.uint64(32)).astype(np.int64)
            it = (buf[2][keep] & np.uint64(0xFFFFFFFF)).astype(np.int64)
            base = t0.min()
            s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # us from the first workgroup's start
            r = {"span": e.max()}
            for code, name in ((0, "integrate"), (1, "cull"), (2, "prep")):
                m = role == code
                if not m.any():
                    continue
                r[name] = [int(m.sum()), s[m].min(), s[m].max(), np.median(e[m]), e[m].max(), (e[m] - s[m]).mean()]
            r["items"] = it[role == 0]
            r["busy"] = (e - s)[role == 0]
            # the CU each workgroup ran on: XCC id and HW_ID bits 8..15 (CU, SH, SE)
            place = buf[3][keep]
            cu = ((place >> np.uint64(32)) << np.uint64(8)) | ((place >> np.uint64(8)) & np.uint64(0xFF))
            r["cu_i"] = cu[role == 0]
            # workgroup b on XCD b % 8 (the dispatch order XCD-aware dealing assumes)?
            b_idx = np.nonzero(keep)[0]
            xcc = (place >> np.uint64(32)).astype(np.int64)
            r["xcc_rr"] = float(np.mean(xcc == (b_idx % 8)))
            r["end_i"] = e[role == 0]
            rows.append(r)
        out = {"world": world, "span_us": round(float(np.mean([r["span"] for r in rows])), 2)}
        for name in ("integrate", "cull", "prep"):
            v = np.array([r[name] for r in rows if name in r])
            if len(v):
                out[name] = {"wgs": int(v[0, 0]), "first_start_us": round(float(v[:, 1].mean()), 2),
                             "last_start_us": round(float(v[:, 2].mean()), 2),
                             "end_median_us": round(float(v[:, 3].mean()), 2),
                             "last_end_us": round(float(v[:, 4].mean()), 2),
                             "busy_mean_us": round(float(v[:, 5].mean()), 2)}
        it = np.concatenate([r["items"] for r in rows])
        out["integrate"]["items_mean"] = round(float(it.mean()), 1)
        busy = rows[-1]["busy"]
        out["integrate"]["busy_deciles_last"] = [round(float(x), 1) for x in np.percentile(busy, range(0, 101, 10))]
        # placement of the last launch's integrate workgroups: how many share a CU, their busy time
        # by that count, and when each CU's last integrate workgroup ends
        cu_i, end_i = rows[-1]["cu_i"], rows[-1]["end_i"]
        ucu, inv, cnt = np.unique(cu_i, return_inverse=True, return_counts=True)
        per = cnt[inv]
        out["integrate"]["cus_by_wgs"] = {str(k): int((cnt == k).sum()) for k in np.unique(cnt)}
        out["integrate"]["busy_by_wgs_per_cu"] = {str(k): round(float(busy[per == k].mean()), 1) for k in np.unique(per)}
        cu_end = np.array([end_i[inv == j].max() for j in range(len(ucu))])
        xcd_of_cu = (ucu >> np.uint64(8)).astype(np.int64)
        out["integrate"]["cu_end_mean_by_xcd"] = {str(x): round(float(cu_end[xcd_of_cu == x].mean()), 1)
                                                  for x in np.unique(xcd_of_cu)}
        out["integrate"]["cu_end_max_by_xcd"] = {str(x): round(float(cu_end[xcd_of_cu == x].max()), 1)
                                                 for x in np.unique(xcd_of_cu)}
        out["xcc_is_wg_mod_8"] = round(float(np.mean([r["xcc_rr"] for r in rows])), 4)
        out["integrate"]["cu_end_deciles"] = [round(float(x), 1) for x in np.percentile(cu_end, range(0, 101, 10))]
        print(json.dumps(out), flush=True)
        del vol


if __name__ == "__main__":
    main()
