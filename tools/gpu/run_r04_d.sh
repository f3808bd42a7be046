# Round 4 call D: GPU tests on the in-tree library (r4g); the hash's launch timeline against the
# dense one (abtest/libwgt.so); the hash driver window with a grown vs a pre-mapped pool; the
# driver-window A/B of the hash's table / volume access (r4e, r4g, tabval, noitemvol).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_d"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$O/tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TSDF_HIP_LIB=$R/abtest/libwgt.so timeout -k 10 300 python -u tools/gpu/wg_times_hash.py > "$O/wg_times_hash.jsonl" 2> "$O/wg_times_hash.err" || exit $?
timeout -k 10 300 python -u tools/gpu/hash_pool_probe.py > "$O/hash_pool.jsonl" 2> "$O/hash_pool.err" || exit $?
for rep in 1 2; do
  for n in r4e r4g tabval noitemvol; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
exit $rc
