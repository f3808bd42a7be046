# VALU issue-cost probe + library A/B on the bench (tools/gpu/run_ab_bench.sh).
set -o pipefail
mkdir -p gpurun_out/probe
hipcc -O3 --offload-arch=gfx950 tools/gpu/valu_probe.hip -o /tmp/valu_probe || exit $?
timeout -k 10 120 /tmp/valu_probe > gpurun_out/probe/valu.txt 2>&1 || exit $?
bash tools/gpu/run_ab_bench.sh "$@"
