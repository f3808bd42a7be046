# Round 4 call C: the whole GPU test suite on the in-tree library, the driver's bench command, then
# the A/B of round-4 builds (run_r04_ab1.sh) -- the A/B also after a failed test, never after a
# crash, a hang or a time limit.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r04_c
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_c/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r04_c/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_c/bench.json 2> gpurun_out/r04_c/bench.err || exit $?
bash tools/gpu/run_r04_ab1.sh || exit $?
exit $rc
