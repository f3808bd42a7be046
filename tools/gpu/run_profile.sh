# Round profile: (1) rocprofv3 --kernel-trace --stats over the default bench command, (2) two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE; --kernel-trace only beside --pmc) over a short
# dense-only bench.  Summaries land in gpurun_out/profile/; tools/summarize_profile.py turns
# them into profiles/.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/profile"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_stats -o run --output-format csv -- python "$R/bench.py" --no-cpu --no-lounge > "$O/bench_under_rocprof.json" 2> "$O/bench_under_rocprof.err" || exit $?
find /tmp/prof_stats -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/pmc_$i -o pmc -- python "$R/bench.py" --steps 50 --warmup 5 --no-hash --no-cpu --no-profile --no-ingest --no-dropin --no-mesh --no-lounge > "$O/pmc_$pass.json" 2> "$O/pmc_$pass.err" || exit $?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "tsdf|Counter_Name" "$f" > "$O/pmc_$pass.csv"
done
