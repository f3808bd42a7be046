# Pipeline event-flag check on rank 0 of the 8-way cyclic shard (TSDF_PIPE_EVFLAGS), with a kernel
# + HIP-API trace to see where the per-batch bubble between integrates comes from.
set -o pipefail
mkdir -p gpurun_out/evf
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
TSDF_PIPE_EVFLAGS=0x20000002 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/p3 -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 1000 --warmup 50 > "$R/gpurun_out/evf/prof.json" 2>&1 || exit $?
find /tmp/p3 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf" "$1" | tail -60 > "$2"' _ {} "$R/gpurun_out/evf/trace_tail.csv" \;
find /tmp/p3 -name "*hip_api_trace.csv" -exec sh -c 'head -1 "$1" > "$2"; tail -400 "$1" >> "$2"' _ {} "$R/gpurun_out/evf/api_tail.csv" \;
