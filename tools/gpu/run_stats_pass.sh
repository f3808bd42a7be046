# rocprofv3 --kernel-trace --stats of the driver's own bench command, unchanged (bench.py --gpus 1
# --steps 20 --warmup 5), and the per-dispatch trace rows of the tsdf kernels (the timed launches
# are picked out by tools/summarize_profile.py).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/profile"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_stats -o run --output-format csv -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench_under_rocprof.json" 2> "$O/bench_under_rocprof.err" || exit $?
find /tmp/prof_stats -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
f=$(find /tmp/prof_stats -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && grep -E "tsdf::|Kernel_Name" "$f" > "$O/kernel_trace_tsdf.csv"
exit 0
