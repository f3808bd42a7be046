set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/gpu/valu_probe > gpurun_out/valu_probe.txt 2>&1 && bash tools/gpu/run_prof_s8.sh
