set -o pipefail
mkdir -p gpurun_out
for a in "" "--depth-f64" "" "--depth-f64"; do
  timeout -k 10 300 python bench.py --no-hash --no-cpu --no-mesh --no-ingest --no-dropin $a > gpurun_out/ab_$RANDOM.json 2>> gpurun_out/ab.err || exit $?
done
grep -h "dense:" gpurun_out/ab.err
