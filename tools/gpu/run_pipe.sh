# Fused three-stage launch (TSDF_PIPELINE=1, default) vs the in-line kernels (=0): GPU tests with
# the in-line path forced, then rank 0 of the 2/4/8-way cyclic shards and the full volume under both.
set -o pipefail
mkdir -p gpurun_out/pipe
TSDF_PIPELINE=1 timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pipe/tests_pipe1.log 2>&1 || exit $?
for p in 0 1; do
  for w in 8:0 4:0 2:0; do
    TSDF_PIPELINE=$p timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > gpurun_out/pipe/s${w%%:*}_$p.json 2> gpurun_out/pipe/s${w%%:*}_$p.err || exit $?
  done
  TSDF_PIPELINE=$p timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu --no-ingest --no-mesh > gpurun_out/pipe/full_$p.json 2> gpurun_out/pipe/full_$p.err || exit $?
done
