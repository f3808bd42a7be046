# Round 3: the owned-brick cull of bucket-range hash shards: GPU tests, then rank 0 of 8 hash
# shards at 512^3 and 1024^3 against the previous library (abtest/libprev.so).
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
O=gpurun_out/owned; mkdir -p $O
for rep in 1 2; do for name in base prev; do
  if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
  timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 > $O/h8_$name.$rep.json 2> $O/h8_$name.$rep.err || exit $?
  timeout -k 10 300 python tools/scaling_sim.py --hash --extent 1024 --only 8:0 --steps 400 > $O/h8k_$name.$rep.json 2> $O/h8k_$name.$rep.err || exit $?
  echo "$name $rep h8(512) $(python -c "import json;print(json.load(open('$O/h8_$name.$rep.json'))['hash8']['fps'])") h8(1024) $(python -c "import json;print(json.load(open('$O/h8k_$name.$rep.json'))['hash8']['fps'])")" >> $O/summary.txt
done; done
cat $O/summary.txt
