# Kernel timeline of rank 0 of an 8-way cyclic shard (pipelined prep/cull).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/prof_s8"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p2 -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 1000 --warmup 50 > "$O/s8.json" 2> "$O/s8.err" || exit $?
find /tmp/p2 -name "*kernel_stats.csv" -exec cp {} "$O/s8_stats.csv" \;
find /tmp/p2 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf|Kernel_Name" "$1" | tail -400 > "$2"' _ {} "$O/s8_trace_tail.csv" \;
