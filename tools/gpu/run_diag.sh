# Work diagnostics of the dense integrate (library built with -DTSDF_DIAG by
# tools/build_variant.sh diag "-DTSDF_DIAG": part x frame pairs computed vs pairs with a valid
# voxel, reported in the probe_steps / lookups counters) on the full volume and an 8-way shard.
set -o pipefail
mkdir -p gpurun_out/diag
for w in 1:0 8:0; do
  TSDF_HIP_LIB=$PWD/abtest/libdiag.so timeout -k 10 300 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > gpurun_out/diag/s${w%%:*}.json 2> gpurun_out/diag/s${w%%:*}.err || exit $?
done
