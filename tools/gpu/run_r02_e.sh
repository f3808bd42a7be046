# VMM probe, GPU tests + smoke, then the dense bench with NZ = 4 and NZ = 8 (TSDF_DENSE_NZ).
set -o pipefail
mkdir -p gpurun_out/nz gpurun_out/probe
hipcc -O2 --offload-arch=gfx950 tools/gpu/vmm_probe.hip -o /tmp/vmm_probe || exit $?
timeout -k 10 60 /tmp/vmm_probe > gpurun_out/probe/vmm.txt 2>&1 || exit $?
bash tools/gpu/run_tests.sh || exit $?
for nz in 4 8; do
  TSDF_DENSE_NZ=$nz timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin --no-lounge > gpurun_out/nz/nz$nz.json 2> gpurun_out/nz/nz$nz.err || exit $?
done
