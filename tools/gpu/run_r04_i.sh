# Round 4 call I: XCD-aware dealing of list items (x1 = in-tree + TSDF_XCD_DEAL=1) and the hash's
# previous 512-thread workgroups (h512) against the in-tree build (cur: 768-thread hash
# workgroups, no prefetch), at the driver window (whole volume, dense + hash) and on rank 0 of
# eighth shards (dense cyclic columns, hash bucket ranges); then the GPU tests of the in-tree build.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_i"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur x1 h512; do
    TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for rep in 1 2; do
  for n in cur x1 h512; do
    echo "$n s8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 48 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$O/tests.log"; exit $rc
