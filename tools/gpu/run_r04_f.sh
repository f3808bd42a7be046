# Round 4 call F: 16-frame launches by default.  The whole GPU test suite, the driver's bench
# command, the driver-window A/B of b16 (the 16-frame build of the previous round-4 kernels)
# against r4k (the in-tree build: next-item prefetch, per-item volume locals), the load-factor
# sweep and the per-frame drop-in rates.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_f"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$O/tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || exit $?
for rep in 1 2; do
  for n in b16 r4k; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
timeout -k 10 400 python -u tools/hash_sweep.py > "$O/hash_sweep.json" 2> "$O/hash_sweep.err" || exit $?
timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 > "$O/dropin.txt" 2> "$O/dropin.err" || exit $?
exit $rc
