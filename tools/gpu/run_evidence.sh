# Round evidence on one GPU: GPU tests + smoke, the default bench line, the rocprofv3 kernel
# stats of the bench and the PMC traffic / SQ passes (tools/summarize_profile.py turns
# gpurun_out/ into profiles/).
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
bash tools/gpu/run_round_prof.sh
