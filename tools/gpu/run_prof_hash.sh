# Kernel-time breakdown of the hash bench (dense skipped via a short run).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/prof_hash"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ph -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-cpu --no-ingest --no-mesh > "$O/b.json" 2> "$O/b.err" || exit $?
find /tmp/ph -name "*kernel_stats.csv" -exec cp {} "$O/stats.csv" \;
