#!/usr/bin/env python3
"""Headline benchmark: depth frames/s (and Mvoxel-updates/s) of 640x480 frames fused into a
512^3 @ 2 cm dense TSDF volume on MI355X, with the voxel-hash path measured on the same frames
(BASELINE.json metric, config[1] "1xMI355X dense grid: 1000 synthetic 640x480 frames into
512^3 @2cm"; config[2] for the hash numbers).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step is one frame integrated (pyramid + fused cull/integrate kernels).  The F synthetic frames
(tsdf_amd.scene: ray-cast room with spheres, u16 millimetre depth, RGB) are generated directly in
HBM before timing; W warmup frames, then K timed frames issued as one asynchronous batch,
bracketed by barrier + synchronize; the max over ranks is taken.  With N ranks each rank owns the
8-voxel x-columns c with c % N == rank (cyclic column shards, DESIGN.md §6: balanced frustum
share per rank) and integrates every frame into them -- no data-path collective -- so total work
is fixed: "scaling": "strong".

Rank 0 prints ONE JSON line.  `roofline` prices the integrate kernel by SURVEY §8(d)'s
algorithmic bytes (24 B per updated voxel + 5 B per pixel per frame) over its HIP-event time;
`cpu_baseline` is the C oracle (oracle/, scalar, one core) on a bounded sample of the same
workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "union-thesis-slam_amd"), os.path.join(REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
ROOM = 10.24
VOXEL = 0.02
PIX = 640 * 480


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000, help="timed frames")
    ap.add_argument("--warmup", type=int, default=100, help="untimed frames")
    ap.add_argument("--frames", type=int, default=1000, help="synthetic frames resident in HBM")
    ap.add_argument("--no-hash", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=5, help="CPU-baseline sample (~2 s per frame)")
    ap.add_argument("--no-profile", action="store_true", help="no HIP events in the timed region")
    ap.add_argument("--no-ingest", action="store_true", help="skip the host-frame (PCIe) measurement")
    ap.add_argument("--ingest-frames", type=int, default=256)
    ap.add_argument("--no-mesh", action="store_true", help="skip the mesh-extraction measurement")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, one GPU per rank) or gloo (rehearsal: several ranks may share a GPU)")
    return ap.parse_args()


def frame_ranges(start, count, F):
    """Split frames [start, start+count) of a cyclic sequence of F frames into contiguous runs."""
    out = []
    while count > 0:
        s = start % F
        n = min(count, F - s)
        out.append((s, n))
        start += n
        count -= n
    return out


def run_timed(vol, depth, rgb, K, Tinv, start, count, F, sync, barrier, profile):
    """Issue `count` frames asynchronously; returns wall seconds (max over ranks)."""
    dptr, cptr = depth.data_ptr(), rgb.data_ptr()
    dstride, cstride = depth[0].numel() * 2, rgb[0].numel()
    hw = tuple(depth.shape[1:3])
    vol.set_profiling(profile)
    vol.stats(reset=True)
    barrier()
    sync()
    t0 = time.perf_counter()
    for s, n in frame_ranges(start, count, F):
        vol.integrate_batch(dptr + s * dstride, cptr + s * cstride, K, Tinv[s:s + n], hw=hw,
                            device_ptrs=True, sync=False)
    vol.sync()
    sync()
    dt = time.perf_counter() - t0
    return dt


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    n = world
    gpu = local if args.dist_backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if n > 1:
        # the backends' connection messages go to fd 1 (gloo prints "Rank r is connected to ...");
        # send them to stderr so that stdout carries only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(args.dist_backend)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    def barrier():
        if n > 1:
            dist.barrier()

    def sync():
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if n == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if n == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    from tsdf_amd import _ffi, grid_fusion, hash_fusion, scene

    # ---- synthetic workload, generated in HBM ---------------------------------------------
    F = args.frames
    t0 = time.perf_counter()
    poses = scene.trajectory(F, seed=0)
    spheres = scene.make_spheres(0)
    depth = torch.empty((F, 480, 640), dtype=torch.int16, device=dev)
    rgb = torch.empty((F, 480, 640, 3), dtype=torch.uint8, device=dev)
    for s in range(0, F, 50):
        d, c = scene.render(poses[s:s + 50], spheres, seed=0, start=s, device=dev, depth_dtype=torch.int16)
        depth[s:s + len(d)] = d
        rgb[s:s + len(c)] = c
    Tinv = np.ascontiguousarray(np.linalg.inv(poses))
    K = scene.intrinsics()
    sync()
    log(f"[rank {rank}] generated {F} frames in HBM in {time.perf_counter() - t0:.1f}s")

    # ---- dense grid: this rank's x-slab of 512^3 @ 2 cm --------------------------------------
    X = int(round(ROOM / VOXEL))
    bnds = np.array([[0.0, ROOM]] * 3)
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):  # the reference-style ctor prints; keep stdout JSON-only
        vol = grid_fusion.TSDFVolume(bnds, VOXEL, device=gpu, shard=(rank, n))
    W, Kt = args.warmup, args.steps
    run_timed(vol, depth, rgb, K, Tinv, 0, W, F, sync, barrier, False)
    dt = run_timed(vol, depth, rgb, K, Tinv, W, Kt, F, sync, barrier, not args.no_profile)
    st = vol.stats()
    dt_max = max_over_ranks(dt)
    vox = sum_over_ranks(float(st["voxel_updates"]))
    fps = Kt / dt_max
    kernel_s = st["kernel_ms"] / 1e3
    # roofline of the integrate kernel on this rank: algorithmic bytes / HIP-event time
    alg_bytes = 24.0 * st["voxel_updates"] + 5.0 * PIX * Kt
    roof = None
    if st["kernel_launches"]:
        ach = alg_bytes / kernel_s / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "tsdf::k_fused<ow==1, NZ=4>: integrates batch k (and culls k+1, preps k+2 "
                          "in the same launch); bytes = batch k's integrate bytes only",
                "kernel_avg_us": round(1e6 * kernel_s / st["kernel_launches"], 2),
                "bytes_per_launch": round(alg_bytes / st["kernel_launches"]),
                "launches": st["kernel_launches"]}
        pmc = os.path.join(REPO, "profiles", "pmc_integrate_r01.json")
        if os.path.exists(pmc):
            with open(pmc) as fh:
                p = json.load(fh)
            roof["traffic"] = p.get("hbm_bytes_per_launch")
            roof["traffic_source"] = "profiles/pmc_integrate_r01.json (separate rocprofv3 --pmc pass)"
    vf_mean = st["voxel_updates"] / Kt
    log(f"[rank {rank}] dense: {Kt} frames in {dt * 1e3:.1f} ms -> {Kt / dt:.0f} frames/s, "
        f"V_f mean {vf_mean:.0f} ({100 * vf_mean / (len(vol.x_index) * X * X):.1f}% of shard), "
        f"kernel {st['kernel_ms']:.1f} ms over {st['kernel_launches']} launches, "
        f"bricks visited/frame {st['bricks_visited'] / Kt:.0f}, touched/frame {st['bricks_touched'] / Kt:.0f}")
    # ---- PCIe-inclusive rate: the same frames from pageable host memory (not `value`) -------
    ingest = None
    if not args.no_ingest:
        ni = min(args.ingest_frames, F)
        dh = depth[:ni].cpu().numpy().view(np.uint16)
        ch = rgb[:ni].cpu().numpy()
        vol.set_profiling(False)
        barrier()
        sync()
        t0 = time.perf_counter()
        vol.integrate_batch(dh, ch, K, Tinv[:ni], sync=True)
        ti = max_over_ranks(time.perf_counter() - t0)
        ingest = {"frames_per_s": round(ni / ti, 1), "frames": ni,
                  "source": "pageable numpy arrays copied by host threads into page-locked bounce "
                            "slots, DMA on a copy stream into four device staging slots, overlapped "
                            "with the pipelined launches (tsdf_dense_integrate_batch without "
                            "TSDF_DEVICE_PTRS)"}
        log(f"[rank {rank}] ingest: {ni} host frames in {ti * 1e3:.1f} ms -> {ni / ti:.0f} frames/s")
    # ---- mesh extraction of the fused volume (not part of `value`) ----
    mesh = None
    if not args.no_mesh and rank == 0:
        import ctypes
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        sync()
        t0 = time.perf_counter()
        _ffi.call("tsdf_dense_extract_mesh", vol._h, ctypes.byref(nv), ctypes.byref(nt))
        tm = time.perf_counter() - t0
        nvox = len(vol.x_index) * X * X
        mesh = {"ms": round(1e3 * tm, 2), "vertices": nv.value, "triangles": nt.value,
                "mvoxels_per_s": round(nvox / tm / 1e6, 1),
                "note": "marching cubes on the device over the rank's shard after the timed run"}
        log(f"[rank {rank}] mesh: {nv.value} vertices, {nt.value} triangles in {tm * 1e3:.1f} ms")
    del vol
    torch.cuda.empty_cache()

    # ---- voxel hash on the same frames (config[2]: 8^3 blocks, 2^22 buckets) ---------------
    hash_res = None
    if not args.no_hash:
        nb = (X // 8) ** 3
        with contextlib.redirect_stdout(sys.stderr):
            ht = hash_fusion.HashTable(np.array([[0.0, ROOM]] * 3), VOXEL, 1 << 22, device=gpu,
                                       max_blocks=nb, shard=rank, n_shards=n)
        run_timed(ht, depth, rgb, K, Tinv, 0, W, F, sync, barrier, False)
        hdt = run_timed(ht, depth, rgb, K, Tinv, W, Kt, F, sync, barrier, not args.no_profile)
        hs = ht.stats()
        info = ht.info()
        if hs["bricks_skipped"]:
            raise RuntimeError(f"hash table/pool overflowed ({hs['bricks_skipped']} bricks skipped)")
        hdt_max = max_over_ranks(hdt)
        hvox = sum_over_ranks(float(hs["voxel_updates"]))
        hash_res = {"frames_per_s": round(Kt / hdt_max, 1),
                    "mvox_updates_per_s": round(hvox / hdt_max / 1e6, 1),
                    "ms_per_frame": round(1e3 * hdt_max / Kt, 4),
                    "buckets": 1 << 22, "block": "8^3",
                    "load_factor": round(sum_over_ranks(info["used"]) / (1 << 22), 4),
                    "blocks_live": int(sum_over_ranks(info["used"])),
                    "mean_probe": round(hs["probe_steps"] / max(1, hs["lookups"]), 3),
                    "max_probe": int(hs["probe_max"]),
                    "kernel_avg_us": round(1e3 * hs["kernel_ms"] / max(1, hs["kernel_launches"]), 2)}
        log(f"[rank {rank}] hash: {Kt / hdt:.0f} frames/s, load {hash_res['load_factor']}")
        del ht

    # ---- CPU baseline: the oracle (C, one core) on a bounded sample -------------------------
    cpu = None
    if rank == 0 and n == 1 and not args.no_cpu:
        import oracle as O
        nfr = max(1, args.cpu_frames)
        ov = O.OracleTSDFVolume(np.array([[0.0, ROOM]] * 3), VOXEL)
        dh = depth[W % F: W % F + nfr].cpu().numpy().view(np.uint16)
        ch = rgb[W % F: W % F + nfr].cpu().numpy()
        t0 = time.perf_counter()
        for i in range(len(dh)):
            ov.integrate(ch[i], dh[i].astype(float) / 1000.0, K, poses[W % F + i])
        ct = time.perf_counter() - t0
        cpu = {"value": round(len(dh) / ct, 4), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{len(dh)} of the synthetic frames into the full 512^3 @ 2 cm volume "
                         f"(oracle/tsdf_oracle.c, full-volume sweep like grid_fusion.py:260-314), "
                         f"{ct:.1f} s",
               "host_cpus": os.cpu_count()}
        log(f"[rank 0] cpu oracle: {len(dh)} frames in {ct:.1f}s")

    if rank == 0:
        line = {
            "metric": "depth frames/sec (640x480 into 512^3 @ 2 cm dense TSDF; hash alongside)",
            "value": round(fps, 1), "unit": "frames/s", "n_gpus": n, "steps": Kt, "warmup": W,
            "ms_per_step": round(1e3 * dt_max / Kt, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (ray-cast 10.24 m room + spheres, u16 mm depth, RGB8; generated in HBM)",
            "config": {"workload": "config[1]: 1000 synthetic 640x480 frames into 512^3 @ 2 cm dense grid",
                       "volume": "512x512x512 @ 0.02 m", "frames_resident": F, "image": "640x480",
                       "parallelism": f"cyclic 8-voxel x-columns over {n} ranks" if n > 1 else "single GPU"},
            "mvox_updates_per_s": round(vox / dt_max / 1e6, 1),
            "mean_voxels_updated_per_frame": round(vox / Kt),
            "hash": hash_res,
            "pcie_inclusive": ingest,
            "mesh": mesh,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if n > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
