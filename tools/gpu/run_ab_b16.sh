# Frames per batch 8 (in-tree) vs 16 (abtest/libb16.so): GPU tests under both, then the quick A/B.
set -o pipefail
mkdir -p gpurun_out/b16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/b16/tests8.log 2>&1 || exit $?
TSDF_HIP_LIB=$PWD/abtest/libb16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/b16/tests16.log 2>&1 || exit $?
bash tools/gpu/run_ab_lib.sh b16
