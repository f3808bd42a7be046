# A/B of the dense integrate variants (TSDF_DENSE_NZ = 1: lane per voxel, frame-parallel
# gathers; 4: z-half waves), tests run under NZ=1.
set -o pipefail
mkdir -p gpurun_out/nz1 gpurun_out/nz4
TSDF_DENSE_NZ=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/nz1/tests.log 2>&1 || exit $?
for nz in 1 4; do
  O=gpurun_out/nz$nz
  for w in 8:0 4:0 2:0; do
    TSDF_DENSE_NZ=$nz timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > $O/s${w%%:*}.json 2> $O/s${w%%:*}.err || exit $?
  done
  TSDF_DENSE_NZ=$nz timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest > $O/full.json 2> $O/full.err || exit $?
done
