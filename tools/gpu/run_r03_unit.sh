# Shard units of 1 / 2 / 4 brick columns (TSDF_SHARD_UNIT): sharded GPU tests with unit 2, then
# the predicted 8-way (and 4-way) strong scaling per unit.
set -o pipefail
mkdir -p gpurun_out/u
TSDF_SHARD_UNIT=2 timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_dist_gpu.py tests/test_mesh_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/u/tests.log 2>&1
for u in 1 2 4; do
  TSDF_SHARD_UNIT=$u timeout -k 10 300 python tools/scaling_sim.py --worlds 1,4,8 > gpurun_out/u/u$u.json 2> gpurun_out/u/u$u.err || exit $?
done
