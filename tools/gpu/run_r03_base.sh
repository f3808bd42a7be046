# Round-3 baseline on a fresh box: GPU tests + smoke, then the default bench line.
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
