# GPU tests + smoke + the bench at the driver's arguments, then the hash load-factor sweep.
set -o pipefail
BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu/run_all.sh || exit $?
mkdir -p gpurun_out/r02c
timeout -k 10 600 python tools/hash_sweep.py > gpurun_out/r02c/hash_sweep.json 2> gpurun_out/r02c/hash_sweep.err
