# Round 3: VALU issue-cost probe, GPU tests + smoke, then the library A/B on the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/gpu/valu_probe > gpurun_out/valu_probe.txt 2>&1 || exit $?
bash tools/gpu/run_tests_ab.sh "$@"
