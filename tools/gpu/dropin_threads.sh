#!/bin/bash
# Per-frame drop-in rate (tools/gpu/dropin_rate.py: 256 per-frame integrate() calls per pass, 5 passes,
# dense and hash) for several copy-pool sizes, each in its own process (the pool is created at the
# first copy and reads TSDF_COPY_THREADS then).  One JSON line per setting into $1.
#   bash tools/gpu/dropin_threads.sh <out.jsonl> [threads ...]
out=$1; shift
for t in "${@:-2 4 6 8}"; do
  TSDF_COPY_THREADS=$t timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 >> "$out" || exit 1
done
