# Round 4 call M: entry words read at item start and stored only when changed (occ: TSDF_OCC_RMW=1)
# against the in-tree build, at the driver window and on the hash eighth shard.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_m"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur occ; do
    TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --kernel-time --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
TSDF_HIP_LIB=$R/abtest/libhdiag.so timeout -k 10 200 python -u tools/gpu/hash_diag.py > "$O/hash_diag.jsonl" 2> "$O/hash_diag.err" || exit $?
TSDF_HIP_LIB=$R/abtest/libocc.so timeout -k 10 600 python -u -m pytest tests/test_hash_gpu.py tests/test_dropin_gpu.py tests/test_long_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests_occ.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$O/tests_occ.log"; exit $rc
