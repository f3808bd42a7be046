# Kernel-time breakdown of (1) the full-volume dense bench and (2) rank 0 of an 8-way cyclic
# shard, to price the per-batch fixed costs (prep, cull, launch gaps) against integrate.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/prof_small"
mkdir -p "$O"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p1 -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-hash --no-cpu > "$O/full.json" 2> "$O/full.err" || exit $?
find /tmp/p1 -name "*kernel_stats.csv" -exec cp {} "$O/full_stats.csv" \;
find /tmp/p1 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf|Kernel_Name" "$1" | tail -400 > "$2"' _ {} "$O/full_trace_tail.csv" \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p2 -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 1000 --warmup 50 > "$O/s8.json" 2> "$O/s8.err" || exit $?
find /tmp/p2 -name "*kernel_stats.csv" -exec cp {} "$O/s8_stats.csv" \;
find /tmp/p2 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf|Kernel_Name" "$1" | tail -400 > "$2"' _ {} "$O/s8_trace_tail.csv" \;
