# Fused three-stage pipeline (default) vs the in-line path (TSDF_PIPELINE=0): GPU tests first,
# then rank 0 of the 8/4/2-way cyclic shards and the full-volume dense bench under both.
set -o pipefail
mkdir -p gpurun_out/fab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fab/tests.log 2>&1 || exit $?
for p in 1 0; do
  for w in 8:0 4:0 2:0; do
    TSDF_PIPELINE=$p timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > gpurun_out/fab/s${w%%:*}_$p.json 2> gpurun_out/fab/s${w%%:*}_$p.err || exit $?
  done
  TSDF_PIPELINE=$p timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-mesh > gpurun_out/fab/full_$p.json 2> gpurun_out/fab/full_$p.err || exit $?
done
