# Quick A/B round: GPU tests, rank 0 of the 8/4/2-way shards, the full dense bench (+ hash).
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
for w in 8:0 4:0 2:0; do
  timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 50 > $O/s${w%%:*}.json 2> $O/s${w%%:*}.err || exit $?
done
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu --no-mesh --no-ingest > $O/full.json 2> $O/full.err || exit $?
