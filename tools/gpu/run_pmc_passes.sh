# The two PMC traffic passes of tools/gpu/run_profile.sh and the SQ pass, without the rocprof stats run.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/profile"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/pmc_$i -o pmc -- python "$R/bench.py" --steps 50 --warmup 5 --no-hash --no-cpu --no-profile --no-ingest --no-dropin --no-mesh --no-lounge > "$O/pmc_$pass.json" 2> "$O/pmc_$pass.err" || exit $?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "tsdf|Counter_Name" "$f" > "$O/pmc_$pass.csv"
done
cd "$R" && bash tools/gpu/run_pmc_sq.sh
