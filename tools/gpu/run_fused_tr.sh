# Fused pipeline: kernel trace of rank 0 of the 8-way shard and of the full-volume bench, and the
# bench with/without the profiling events (their fence flags: TSDF_PROF_EVFLAGS).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ftr
mkdir -p $O
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-mesh --no-ingest > $O/full_prof.json 2> $O/full_prof.err || exit $?
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-mesh --no-ingest --no-profile > $O/full_noprof.json 2> $O/full_noprof.err || exit $?
TSDF_PROF_EVFLAGS=0 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-mesh --no-ingest > $O/full_prof_fence.json 2> $O/full_prof_fence.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p5 -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 1000 --warmup 50 > $O/s8.json 2> $O/s8.err || exit $?
find /tmp/p5 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf" "$1" | tail -60 > "$2"' _ {} "$O/s8_trace.csv" \;
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p6 -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-hash --no-cpu --no-mesh --no-ingest > $O/full_tr.json 2> $O/full_tr.err || exit $?
find /tmp/p6 -name "*kernel_trace.csv" -exec sh -c 'grep -E "tsdf" "$1" | tail -60 > "$2"' _ {} "$O/full_trace.csv" \;
