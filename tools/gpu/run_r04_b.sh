# Round 4 call B: the clock-ramp experiment, then the whole GPU test suite on the in-tree library.
set -o pipefail
R=$(pwd)
bash tools/gpu/run_r04_clock.sh || exit $?
cd "$R"
mkdir -p gpurun_out/r04_b
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_b/tests.log 2>&1 || exit $?
