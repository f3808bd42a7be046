# Hash load-factor sweep (tools/hash_sweep.py) on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/hash_sweep.py > gpurun_out/hash_sweep.json 2> gpurun_out/hash_sweep.err
