# GPU round trip: parity tests, smoke, bench (+ rocprofv3 kernel stats).  Stops at the first
# step that fails in a way that may have hurt the GPU.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ -n "${SCALE:-}" ]; then
  timeout -k 10 600 python tools/scaling_sim.py > gpurun_out/scaling_sim.json 2> gpurun_out/scaling_sim.err
  rc=$?; echo "scaling rc=$rc" >> gpurun_out/scaling_sim.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-cpu --no-profile > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
  rc=$?
  mkdir -p "$R/gpurun_out/prof"
  find /tmp/prof -name "*stats*.csv" -exec cp {} "$R/gpurun_out/prof/" \;
  exit $rc
fi
