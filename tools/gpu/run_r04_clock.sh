# Is the driver window's deficit a clock ramp?  The driver's bench command under rocprofv3 kernel
# traces, plain and with 300 ms of untimed integrate work first (--preheat-ms), twice each,
# alternating; the dense leg only.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_clock"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for ph in 0 300; do
    rm -rf /tmp/pc
    timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pc -o run --output-format csv -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --no-lounge --no-hash --no-dropin --no-mesh --no-ingest --preheat-ms $ph > "$O/bench_ph${ph}_$rep.json" 2> "$O/bench_ph${ph}_$rep.err" || exit $?
    f=$(find /tmp/pc -name "*kernel_trace.csv" | head -1)
    grep -E "k_fused<true, 4, 0>|Kernel_Name" "$f" > "$O/trace_ph${ph}_$rep.csv"
  done
done
# and without the profiler (the plain numbers)
cd "$R"
for rep in 1 2; do
  for ph in 0 300; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-lounge --no-hash --no-dropin --no-mesh --no-ingest --preheat-ms $ph >> "$O/plain.jsonl" 2>> "$O/plain.err" || exit $?
  done
done
