# A/B of library builds: the in-tree library and abtest/lib<name>.so for each name given
# (TSDF_HIP_LIB), quick set each (tools/gpu/run_ab_quick.sh layout under gpurun_out/ab_<name>).
set -o pipefail
for name in base "$@"; do
  O=gpurun_out/ab_$name
  mkdir -p $O
  if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
  timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
  for w in 8:0 4:0 2:0; do
    timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > $O/s${w%%:*}.json 2> $O/s${w%%:*}.err || exit $?
  done
  timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest > $O/full.json 2> $O/full.err || exit $?
done
