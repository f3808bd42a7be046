# Work diagnostics of the dense integrate (library built with -DTSDF_DIAG: brick-part x frame
# pairs computed vs pairs with a valid voxel, in the probe_steps / lookups counters).
set -o pipefail
mkdir -p gpurun_out/diag
for w in 1:0 8:0; do
  TSDF_HIP_LIB=$PWD/tools/gpu/libtsdf_diag.so timeout -k 10 300 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > gpurun_out/diag/s${w%%:*}.json 2> gpurun_out/diag/s${w%%:*}.err || exit $?
done
