# A/B: dense-only bench with the in-tree library (A) and abtest/libB.so (B), after the GPU tests.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
for v in A B; do
  if [ $v = B ]; then export TSDF_HIP_LIB=$(pwd)/abtest/libB.so; fi
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-hash --no-cpu > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit $?
done
