# Predicted 8-way strong scaling with 8 vs 16 frames per batch (abtest/libb16.so, built by
# tools/build_variant.sh b16 "-DTSDF_MAX_BATCH=16").
set -o pipefail
mkdir -p gpurun_out/b16s
timeout -k 10 300 python tools/scaling_sim.py --worlds 1,8 > gpurun_out/b16s/b8.json 2> gpurun_out/b16s/b8.err || exit $?
TSDF_HIP_LIB=$PWD/abtest/libb16.so timeout -k 10 300 python tools/scaling_sim.py --worlds 1,8 > gpurun_out/b16s/b16.json 2> gpurun_out/b16s/b16.err || exit $?
