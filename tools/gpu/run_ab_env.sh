# A/B of environment settings on the in-tree library: each argument is "name:VAR=value[,VAR=value]"
# (tools/show_ab.sh gpurun_out/ab_<name>).
set -o pipefail
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  O=gpurun_out/ab_$name
  mkdir -p $O
  (
    for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
    for w in 8:0 4:0 2:0; do
      timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > $O/s${w%%:*}.json 2> $O/s${w%%:*}.err || exit $?
    done
    timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest --no-hash > $O/full.json 2> $O/full.err || exit $?
  ) || exit $?
done
