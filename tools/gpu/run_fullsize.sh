set -o pipefail
mkdir -p gpurun_out/ft
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k full_size > gpurun_out/ft/test.log 2>&1 || exit $?
bash tools/gpu/run_inline_prof.sh
