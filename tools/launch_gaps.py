"""Per-launch duration and the gap to the next launch of one kernel from a rocprofv3
--kernel-trace CSV (tools/gpu/run_gaps.sh):  python tools/launch_gaps.py trace.csv [name-substring]"""
import csv
import sys

import numpy as np


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_fused"
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    s = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
    e = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
    o = np.argsort(s)
    s, e = s[o], e[o]
    dur = (e - s) / 1e3
    gap = (s[1:] - e[:-1]) / 1e3
    gap = gap[gap < 50]  # consecutive launches of one call (not the host's pauses between calls)
    print(f"{sub}: {len(s)} launches, duration median {np.median(dur):.2f} us (p10 {np.percentile(dur, 10):.2f}, "
          f"p90 {np.percentile(dur, 90):.2f}); gap to the next launch median {np.median(gap):.2f} us "
          f"(p10 {np.percentile(gap, 10):.2f}, p90 {np.percentile(gap, 90):.2f}, n {len(gap)})")


if __name__ == "__main__":
    main()
