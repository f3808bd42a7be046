set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-cpu --no-profile > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
rc=$?
mkdir -p "$R/gpurun_out/prof"
find /tmp/prof -name "*stats*.csv" -exec cp {} "$R/gpurun_out/prof/" \;
ls -laR /tmp/prof > "$R/gpurun_out/prof/listing.txt"
exit $rc
