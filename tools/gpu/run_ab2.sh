# A/B (in-tree library vs abtest/libB.so): GPU tests, full-volume dense+hash bench and the 8-way
# shard's rank 0, for each library.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 240 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
for v in A B; do
  if [ $v = B ]; then export TSDF_HIP_LIB=$(pwd)/abtest/libB.so; fi
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-ingest > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit $?
  timeout -k 10 300 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 50 > gpurun_out/ab/s8_$v.json 2> gpurun_out/ab/s8_$v.err || exit $?
done
