# Launch-wide work queue (integrate_items): GPU tests, then bench + eighth-shard rank 0 for the
# in-tree library (chunk 2) and abtest/lib{static,f8,f14,c1,c4}.so, interleaved twice; per-workgroup
# times with the queue (abtest/libwgt2.so).
set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_dropin_gpu.py tests/test_hash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/tests.log 2>&1 || exit $?
TSDF_HIP_LIB=$PWD/abtest/libwgt2.so timeout -k 10 240 python -u tools/gpu/wg_times.py > gpurun_out/q/wg_times.txt 2>&1 || exit $?
for rep in 1 2; do
  for name in base static f8 f14 c1 c4; do
    if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin > gpurun_out/q/$name.$rep.json 2> gpurun_out/q/$name.$rep.err || exit $?
    timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 50 > gpurun_out/q/s8_$name.$rep.json 2> gpurun_out/q/s8_$name.$rep.err || exit $?
    echo "$name $rep $(grep -h 'dense:' gpurun_out/q/$name.$rep.err | sed 's/.*-> //;s/ frames.*//') $(grep -h 'hash:' gpurun_out/q/$name.$rep.err | sed 's/.*hash: //;s/ frames.*//') s8 $(python -c "import json;print(json.load(open('gpurun_out/q/s8_$name.$rep.json'))['fps'])")" >> gpurun_out/q/summary.txt
  done
done
cat gpurun_out/q/summary.txt
