# Dense NZ=8 (one wave per brick) at 4 waves/SIMD vs the default NZ=4 at 6 waves/SIMD.
set -o pipefail
mkdir -p gpurun_out/nz
TSDF_HIP_LIB=$PWD/abtest/libw4.so TSDF_DENSE_NZ=8 timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin --no-lounge --no-hash > gpurun_out/nz/w4nz8.json 2> gpurun_out/nz/w4nz8.err || exit $?
TSDF_HIP_LIB=$PWD/abtest/libw4.so TSDF_DENSE_NZ=4 timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin --no-lounge --no-hash > gpurun_out/nz/w4nz4.json 2> gpurun_out/nz/w4nz4.err || exit $?
grep -h "dense:" gpurun_out/nz/w4*.err
