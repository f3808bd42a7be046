# GPU tests + smoke, then the dense bench with NZ = 4 and NZ = 8 (TSDF_DENSE_NZ) and the hash leg.
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
mkdir -p gpurun_out/nz
for nz in 4 8; do
  TSDF_DENSE_NZ=$nz timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin --no-lounge > gpurun_out/nz/nz$nz.json 2> gpurun_out/nz/nz$nz.err || exit $?
done
grep -h "dense:\|hash:" gpurun_out/nz/*.err
