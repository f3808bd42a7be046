# Round 4: the driver-window diagnosis (tools/gpu/window_probe.py) and a per-dispatch kernel trace
# of the driver's own bench command.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_window"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 300 python -u tools/gpu/window_probe.py > "$O/window_probe.jsonl" 2> "$O/window_probe.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_drv -o run --output-format csv -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu > "$O/bench_driver_args.json" 2> "$O/bench_driver_args.err" || exit $?
find /tmp/prof_drv -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
# the trace rows of the tsdf kernels only (the whole trace is >100 MB of torch's own kernels)
f=$(find /tmp/prof_drv -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && grep -E "tsdf::|Kernel_Name" "$f" > "$O/kernel_trace_tsdf.csv"
ls -la "$O"
cd "$R"
# bench.py --gpus 2 on a one-GPU box: two ranks it launches itself, sharing the GPU over gloo
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-hash --no-cpu --no-dropin --no-lounge > "$O/bench_gpus2_gloo.json" 2> "$O/bench_gpus2_gloo.err" || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests_hash.log" 2>&1 || exit $?
