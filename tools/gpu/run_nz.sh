# A/B of the dense integrate's z-split (TSDF_DENSE_NZ = 8 | 4): tests with the default, then the
# full-volume bench and the 8-way shard rank 0 under each setting.
set -o pipefail
mkdir -p gpurun_out/nz
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
for nz in 8 4; do
  TSDF_DENSE_NZ=$nz timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-ingest > gpurun_out/nz/full$nz.json 2> gpurun_out/nz/full$nz.err || exit $?
  TSDF_DENSE_NZ=$nz timeout -k 10 300 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 50 > gpurun_out/nz/s8_$nz.json 2> gpurun_out/nz/s8_$nz.err || exit $?
done
