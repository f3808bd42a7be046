#!/usr/bin/env python3
"""Turn gpurun_out/profile/ and gpurun_out/pmc_sq/ (tools/gpu/run_round_prof.sh) into the committed
profile summaries, each stamped with the build id of the library that ran (tsdf_build_id, from the
bench line printed under the profiler):
  profiles/<tag>_kernel_stats.csv      rocprofv3 --kernel-trace --stats of the driver's bench command
  profiles/<tag>_bench.json            the bench line printed under that profiler
  profiles/<tag>_timed_launches.csv    the trace rows of the 20 timed integrate launches, and their
                                       average (must agree with the line's roofline.kernel_avg_us)
  profiles/pmc_integrate_<tag>.json    HBM traffic per timed integrate launch (FETCH_SIZE/WRITE_SIZE)
  profiles/pmc_sq_<tag>.json           SQ issue counters per timed integrate launch
  profiles/pmc_hash_<tag>.json         the same counters (traffic + SQ) of the hash launch
                                       k_fused_hash<0, true> in the bench's inserting hash window (and,
                                       as a second block, in its no-allocation repeat window)

The timed launches: every bench.py call of n batches issues n + 2 pipelined launches of
k_fused<true, 4, 0, true> (the cold window, the clock warm-up, the W warm-up steps, then the timed call,
whose first two launches fill the pipeline); the bench line records the dispatch-order index of
the first timed integrate launch (roofline.first_timed_launch_index), and the K launches from it
are the timed ones.

FETCH_SIZE/WRITE_SIZE are KiB.  FETCH_SIZE on gfx950 is (TCC_BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64
+ RDREQ_32B*32) (rocprofiler-sdk counter_defs.yaml): a 128-B memory-side read request is tallied at 64 B,
the guide's "half of a wide streaming read".  Every L2 fill is such a request whatever the access
width -- 2- and 4-byte gathers included (tools/gpu/fetch_probe.hip, profiles/r06_fetch_probe/) -- so
the tally is half of this kernel's reads, gathers and state loads alike; the RDREQ pass counts the
L2's memory-side read requests by size (TCC_EA0_RDREQ_32B / _64B / _128B) and the read bytes are
32*n32 + 64*n64 + 128*n128, without assuming it.  WRITE_SIZE is exact for 16-B/lane stores.  Both
count L2 memory-side traffic: Infinity-Cache hits included, so an upper bound on DRAM bytes.
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the bench's integrate launches (CU = true: u32 colour registers, the canonical volume); DK = 2 is
# the texel variant the host picks for handles of >= 2^17 bricks (Base::texel_for), DK = 0 the
# two-gather one (older builds, TSDF_TEXEL=0).  use_kernels() picks the one a profile holds.
KERNELS = ("tsdf::k_fused<true, 4, 2, true>", "tsdf::k_fused<true, 4, 0, true>")
HASH_KERNELS = ("k_fused_hash<2, true>", "k_fused_hash<0, true>")
KERNEL, HASH_KERNEL = KERNELS[0], HASH_KERNELS[0]
W, K = 5, 20  # the driver's --warmup / --steps


def use_kernels(csv_path):
    """Set KERNEL / HASH_KERNEL to the variants the profile's rows name (texel variant first)."""
    global KERNEL, HASH_KERNEL
    with open(csv_path) as f:
        text = f.read()
    KERNEL = next((k for k in KERNELS if k in text), KERNELS[0])
    HASH_KERNEL = next((k for k in HASH_KERNELS if k in text), HASH_KERNELS[0])


def bench_line(path):
    with open(path) as f:
        return json.loads([l for l in f if l.startswith("{")][-1])


def first_index(line):
    """The bench line's first_timed_launch_index (top level, or in its roofline block); None for a
    line without it (a pass run with --no-profile before bench.py printed it at top level)."""
    if line.get("first_timed_launch_index") is not None:
        return line["first_timed_launch_index"]
    return (line.get("roofline") or {}).get("first_timed_launch_index")


def timed(rows_by_dispatch, first):
    """rows_by_dispatch: [(dispatch_id, row)] of KERNEL -> the K timed launches, from the index the
    bench line records.  first None: the dense-only PMC / SQ passes end with the timed call, so its
    K integrate launches are the process's last K launches of KERNEL (checked by pmc_timed: the two
    launches before them are the call's pipeline-fill launches, prep / cull only)."""
    rows = sorted(rows_by_dispatch, key=lambda r: r[0])
    if first is None:
        first = len(rows) - K
    return rows[first:first + K]


def pmc_timed(path, counter, first, ids=None):
    """The counter's values on the K timed launches (summed over dimensions / XCDs); ids: take
    exactly these dispatches (the timed set found on another counter of the same pass)."""
    use_kernels(path)
    per = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or KERNEL not in row["Kernel_Name"]:
            continue
        d = int(row["Dispatch_Id"])
        per[d] = per.get(d, 0.0) + float(row["Counter_Value"])  # (summed over dimensions / XCDs)
    if ids is not None:
        return [per[d] for d in ids]
    t = timed(list(per.items()), first)
    if first is None:  # the two launches before the last K must be the pipeline fill (no integrate)
        rows = sorted(per.items())
        fill = [v for _, v in rows[-K - 2:-K]]
        med = statistics.median(v for _, v in t)
        if len(fill) != 2 or max(fill) > 0.1 * med:
            raise RuntimeError(f"{path}: the last {K} launches of {KERNEL} are not the timed call")
    return [v for _, v in t]


RDREQ = ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"]


def counter_rows(path, kernel):
    """{dispatch: {counter: value summed over dimensions}} of one kernel in a pmc csv."""
    per = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def request_bytes(m):
    """Read bytes from the request counts by size, and the requests the sizes do not cover."""
    n32, n64, n128 = (m.get(c, 0.0) for c in RDREQ[1:])
    return {"rdreq": m.get(RDREQ[0]), "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
            "read_bytes_by_request_size": 32 * n32 + 64 * n64 + 128 * n128,
            "requests_unsized": (m.get(RDREQ[0]) or 0.0) - n32 - n64 - n128}


def main(tag):
    src = os.path.join(REPO, "gpurun_out", "profile")
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    use_kernels(os.path.join(src, "kernel_trace_tsdf.csv"))
    shutil.copy(os.path.join(src, "kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    line = bench_line(os.path.join(src, "bench_under_rocprof.json"))
    with open(os.path.join(dst, f"{tag}_bench.json"), "w") as f:
        f.write(json.dumps(line) + "\n")
    bid = line.get("build_id")
    # the timed launches' trace rows
    trace = [r for r in csv.DictReader(open(os.path.join(src, "kernel_trace_tsdf.csv")))
             if KERNEL in r["Kernel_Name"]]
    t = timed([(int(r["Dispatch_Id"]), r) for r in trace], first_index(line))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for _, r in t]
    with open(os.path.join(dst, f"{tag}_timed_launches.csv"), "w") as f:
        f.write(f"# {KERNEL}: the {K} timed integrate launches of bench.py --gpus 1 --steps {K} --warmup {W} "
                f"under rocprofv3 (build {bid}); average {statistics.mean(durs):.2f} us, the line's "
                f"roofline.kernel_avg_us {line['roofline']['kernel_avg_us']} (HIP events)\n")
        f.write("dispatch_id,start_ns,end_ns,duration_us\n")
        for (d, r), us in zip(t, durs):
            f.write(f"{d},{r['Start_Timestamp']},{r['End_Timestamp']},{us:.2f}\n")
    pl = bench_line(os.path.join(src, "pmc_FETCH_SIZE.json"))
    pw = bench_line(os.path.join(src, "pmc_WRITE_SIZE.json"))
    fetch = pmc_timed(os.path.join(src, "pmc_FETCH_SIZE.csv"), "FETCH_SIZE", first_index(pl))
    write = pmc_timed(os.path.join(src, "pmc_WRITE_SIZE.csv"), "WRITE_SIZE", first_index(pw))
    pr = bench_line(os.path.join(src, "pmc_RDREQ.json"))
    per = counter_rows(os.path.join(src, "pmc_RDREQ.csv"), KERNEL)
    ids = [d for d, _ in timed([(d, m.get(RDREQ[0], 0.0)) for d, m in per.items()], first_index(pr))]
    reqs = [request_bytes(per[d]) for d in ids]
    sys.path.insert(0, REPO)
    import bench
    fk = statistics.median(fetch) * 1024.0
    wk = statistics.median(write) * 1024.0
    rb = statistics.median(r["read_bytes_by_request_size"] for r in reqs)
    summary = {"kernel": KERNEL, "build_id": pl.get("build_id"), "workload": bench.WORKLOAD,
               "window": f"bench.py --gpus 1 --steps {K} --warmup {W}: the {K} timed launches (median)",
               "launches_sampled": [len(fetch), len(write), len(reqs)],
               "fetch_size_bytes_raw": fk, "write_bytes": wk,
               "read_requests_median": {k: statistics.median(r[k] for r in reqs) for k in reqs[0]},
               "read_bytes": rb,
               "l2_memside_bytes_per_launch": round(rb + wk),
               "raw_bytes_per_launch": round(fk + wk),
               "timed_launch_avg_us_under_rocprof": round(statistics.mean(durs), 2),
               "build_ids": {"FETCH_SIZE": pl.get("build_id"), "WRITE_SIZE": pw.get("build_id"),
                             "RDREQ": pr.get("build_id")},
               "note": " ".join(l.strip() for l in __doc__.strip().splitlines()[-8:])}
    with open(os.path.join(dst, f"pmc_integrate_{tag}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


def sq(tag):
    """gpurun_out/pmc_sq/pmc_sq.csv (tools/gpu/run_pmc_sq.sh) -> profiles/pmc_sq_<tag>.json: SQ
    counters per timed launch of the dense integrate launch and its VALU-busy fraction."""
    src = os.path.join(REPO, "gpurun_out", "pmc_sq")
    use_kernels(os.path.join(src, "pmc_sq.csv"))
    names = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
             "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_VMEM", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]
    pl = bench_line(os.path.join(src, "bench.json"))
    first = first_index(pl)
    # the timed dispatches, found on the VALU instruction count (the fill launches have almost none)
    per = {}
    for row in csv.DictReader(open(os.path.join(src, "pmc_sq.csv"))):
        if row["Counter_Name"] == "SQ_INSTS_VALU" and KERNEL in row["Kernel_Name"]:
            per[int(row["Dispatch_Id"])] = per.get(int(row["Dispatch_Id"]), 0.0) + float(row["Counter_Value"])
    pmc_timed(os.path.join(src, "pmc_sq.csv"), "SQ_INSTS_VALU", first)  # (checks the fill launches)
    ids = [d for d, _ in timed(list(per.items()), first)]
    med = {c: statistics.median(pmc_timed(os.path.join(src, "pmc_sq.csv"), c, first, ids)) for c in names}
    sys.path.insert(0, REPO)
    import bench
    out = {"kernel": KERNEL, "build_id": pl.get("build_id"), "median_per_launch": med,
           # SQ_* cycle counters count quad-cycles; 1024 SIMDs, GRBM_GUI_ACTIVE summed over 8 XCDs
           "valu_busy_per_simd": round(med["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * med["GRBM_GUI_ACTIVE"] / 8), 3),
           "valu_per_vmem": round(med["SQ_INSTS_VALU"] / med["SQ_INSTS_VMEM"], 1),
           "wait_any_frac": round(med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"], 3),
           "workload": bench.WORKLOAD,
           "window": f"bench.py --gpus 1 --steps {K} --warmup {W}: the {K} timed launches (median)",
           "note": "rocprofv3 --pmc pass (tools/gpu/run_pmc_sq.sh); SQ_* cycle counters in quad-cycles per "
                   "MI355X_MICROARCH.md; busy = ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)"}
    with open(os.path.join(REPO, "profiles", f"pmc_sq_{tag}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


SQ_NAMES = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_VMEM", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def hash_windows(path):
    """Per-dispatch counters of HASH_KERNEL in one pass -> (inserting window, repeat window):
    the hash leg ends with the timed call (K + 2 launches: two pipeline fills, then K integrating)
    and the no-allocation repeat (K + 2 more), the process's last 2 (K + 2) launches of the kernel."""
    use_kernels(path)
    per = {}
    for r in csv.DictReader(open(path)):
        if HASH_KERNEL not in r["Kernel_Name"]:
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = [per[k] for k in sorted(per)][-2 * (K + 2):]
    if len(rows) != 2 * (K + 2):
        raise RuntimeError(f"{path}: {len(rows)} hash launches, expected {2 * (K + 2)}")
    return rows[2:K + 2], rows[K + 4:]


def hash_profile(tag):
    """profile/pmc_{FETCH,WRITE}_SIZE.csv and pmc_sq/pmc_sq.csv -> profiles/pmc_hash_<tag>.json."""
    src = os.path.join(REPO, "gpurun_out", "profile")
    use_kernels(os.path.join(src, "pmc_FETCH_SIZE.csv"))
    sys.path.insert(0, REPO)
    import bench
    out = {"kernel": "tsdf::" + HASH_KERNEL, "workload": bench.HASH_WORKLOAD,
           "window": f"bench.py --gpus 1 --steps {K} --warmup {W}, hash leg: the {K} timed launches of the "
                     "inserting window (median); no_alloc_repeat: the same window again"}
    blocks = {"inserting": {}, "no_alloc_repeat": {}}
    for path, names in ((os.path.join(src, "pmc_FETCH_SIZE.csv"), ["FETCH_SIZE"]),
                        (os.path.join(src, "pmc_WRITE_SIZE.csv"), ["WRITE_SIZE"]),
                        (os.path.join(src, "pmc_RDREQ.csv"), RDREQ),
                        (os.path.join(REPO, "gpurun_out", "pmc_sq", "pmc_sq.csv"), SQ_NAMES)):
        ins, rep = hash_windows(path)
        for key, rows in (("inserting", ins), ("no_alloc_repeat", rep)):
            for n in names:
                blocks[key][n] = statistics.median(r[n] for r in rows)
    for key, m in blocks.items():
        m.update(request_bytes(m))
        m["raw_bytes"] = round(1024 * (m["FETCH_SIZE"] + m["WRITE_SIZE"]))
        m["l2_memside_bytes"] = round(m["read_bytes_by_request_size"] + 1024 * m["WRITE_SIZE"])
        m["valu_busy_per_simd"] = round(m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
        m["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    ins = blocks["inserting"]
    out["build_id"] = bench_line(os.path.join(src, "pmc_FETCH_SIZE.json")).get("build_id")
    out["l2_memside_bytes_per_launch"] = ins["l2_memside_bytes"]
    out["raw_bytes_per_launch"] = ins["raw_bytes"]
    out["median_per_launch"] = {n: ins[n] for n in SQ_NAMES}
    out["valu_busy_per_simd"] = ins["valu_busy_per_simd"]
    out["wait_any_frac"] = ins["wait_any_frac"]
    out["no_alloc_repeat"] = blocks["no_alloc_repeat"]
    out["note"] = ("read bytes from the L2's memory-side read requests by size (32/64/128 B, as pmc_integrate_*; "
                   "FETCH_SIZE tallies a 128-B request at 64 B); SQ cycle counters in quad-cycles; "
                   "busy = ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)")
    with open(os.path.join(REPO, "profiles", f"pmc_hash_{tag}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sq":
        sq(*sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "hash":
        hash_profile(*sys.argv[2:])
    else:
        main(*sys.argv[1:])
