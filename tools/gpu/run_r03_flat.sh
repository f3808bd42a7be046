# Round 3: cull without the superbrick level (abtest/libflat.so) against the in-tree library:
# bench (dense, hash), dense and hash eighth shards, half / quarter dense shards.
set -o pipefail
bash tools/gpu/ab.sh gpurun_out/flat 2 base flat || exit $?
for rep in 1 2; do for name in base flat; do for w in 2 4; do
  if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
  timeout -k 10 200 python tools/scaling_sim.py --only $w:0 --steps 1000 --warmup 50 > gpurun_out/flat/w${w}_$name.$rep.json 2>/dev/null || exit $?
  echo "w$w $name $rep $(python -c "import json;print(json.load(open('gpurun_out/flat/w${w}_$name.$rep.json'))['fps'])")" >> gpurun_out/flat/shards.txt
done; done; done
cat gpurun_out/flat/shards.txt
