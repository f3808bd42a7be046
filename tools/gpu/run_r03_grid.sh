# More integrate workgroups than resident slots (TSDF_GRID_Q quarters; static dealing): bench +
# eighth-shard rank 0 for abtest/lib{static,g6,g8,g12,g16}.so interleaved twice, and the
# per-workgroup times of g8 (abtest/libwg8.so).
set -o pipefail
mkdir -p gpurun_out/g
WG_DUMP=1 TSDF_HIP_LIB=$PWD/abtest/libwg8.so timeout -k 10 240 python -u tools/gpu/wg_times.py > gpurun_out/g/wg_times.txt 2>&1 || exit $?
for rep in 1 2; do
  for name in static g6 g8 g12 g16; do
    export TSDF_HIP_LIB=$PWD/abtest/lib$name.so
    timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin > gpurun_out/g/$name.$rep.json 2> gpurun_out/g/$name.$rep.err || exit $?
    timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 50 > gpurun_out/g/s8_$name.$rep.json 2> gpurun_out/g/s8_$name.$rep.err || exit $?
    echo "$name $rep $(grep -h 'dense:' gpurun_out/g/$name.$rep.err | sed 's/.*-> //;s/ frames.*//') $(grep -h 'hash:' gpurun_out/g/$name.$rep.err | sed 's/.*hash: //;s/ frames.*//') s8 $(python -c "import json;print(json.load(open('gpurun_out/g/s8_$name.$rep.json'))['fps'])")" >> gpurun_out/g/summary.txt
  done
done
cat gpurun_out/g/summary.txt
