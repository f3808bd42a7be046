# Hash fused launch vs in-line (TSDF_PIPELINE=0): all GPU tests under the default, then the bench
# (dense + hash) under both settings.
set -o pipefail
O=gpurun_out/abh
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest > $O/fused.json 2> $O/fused.err || exit $?
TSDF_PIPELINE=0 timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest > $O/inline.json 2> $O/inline.err || exit $?
