# A/B of library builds on one rank's shard of the 8- and 4-GPU runs (tools/scaling_sim.py --only):
# the in-tree library ("base") and abtest/lib<name>.so, interleaved twice.
set -o pipefail
mkdir -p gpurun_out/abs
for rep in 1 2; do
  for name in base "$@"; do
    if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
    for o in 8:0 4:0; do
      timeout -k 10 300 python tools/scaling_sim.py --only $o --steps 400 --warmup 24 > gpurun_out/abs/$name.$o.$rep.json 2> gpurun_out/abs/$name.$o.$rep.err || exit $?
      echo "$name $rep $o $(python -c "import json;print(json.loads(open('gpurun_out/abs/$name.$o.$rep.json').read().strip().splitlines()[-1])['fps'])")" >> gpurun_out/abs/summary.txt
    done
  done
done
cat gpurun_out/abs/summary.txt
