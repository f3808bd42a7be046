# The rocprofv3 --kernel-trace --stats pass of tools/gpu/run_profile.sh alone (the bench without
# the CPU baseline and without the lounge leg, whose small-volume launches are the same kernel
# instance as the 512^3 integrate and would mix into its average).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/profile"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_stats -o run --output-format csv -- python "$R/bench.py" --no-cpu --no-lounge > "$O/bench_under_rocprof.json" 2> "$O/bench_under_rocprof.err" || exit $?
find /tmp/prof_stats -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
