#!/usr/bin/env python3
"""gpurun_out/r04_v (tools/gpu/run_r04_v.sh) -> profiles/r04_v/hash_pmc.json: per-launch medians of
the hash launch's counters in the bench's two hash windows.  The hash leg ends with the timed call
(22 launches: 2 pipeline-fill + 20 integrating, the window that inserts) and the no-allocation
repeat (22 more); they are the process's last 44 launches of k_fused_hash<0>."""
import csv
import json
import os
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "r04_v")
KERNEL = "k_fused_hash<0>"


def per_dispatch(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        d = out.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    res = {"kernel": "tsdf::" + KERNEL, "window": "bench.py hash leg at --steps 20 --warmup 5 (rocprofv3 --pmc passes)"}
    for i in (1, 2, 3):
        rows = per_dispatch(os.path.join(SRC, f"pass{i}.csv"))[-44:]
        ins, rep = rows[2:22], rows[24:44]
        for name in rows[-1]:
            res.setdefault("inserting", {})[name] = statistics.median(r[name] for r in ins)
            res.setdefault("no_alloc_repeat", {})[name] = statistics.median(r[name] for r in rep)
    for k in ("inserting", "no_alloc_repeat"):
        m = res[k]
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes"] = round(1024 * (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]))
        if "SQ_ACTIVE_INST_VALU" in m:
            m["valu_busy_per_simd"] = round(m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
            m["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    os.makedirs(os.path.join(REPO, "profiles", "r04_v"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r04_v", "hash_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
