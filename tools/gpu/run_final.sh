# Round 3 final evidence on the committed kernels: GPU tests + smoke, the default bench line and
# the rocprofv3 kernel stats of the bench (the PMC passes of profiles/pmc_*_r03.json ran on the
# commit before the flat cull).
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
bash tools/gpu/run_stats_pass.sh
