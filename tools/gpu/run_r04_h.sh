# Round 4 call H: the async table-growth fix (tests + the load-factor sweep), the item / claim-word
# prefetch A/B (cur = in-tree with both; p0 = no item prefetch; p0r0 = neither; b16 = commit
# 42cd0e2 at 16 frames), hash workgroup shapes (p0w768: 768-thread hash workgroups; p0hw5: 5
# waves/SIMD), and the hash pool on mapped ranges against plain allocations.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_h2"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
# (the tests and the pre-fix control ran in the first attempt: gpurun_out/r04_h/tests*.txt)
timeout -k 10 500 python -u tools/hash_sweep.py > "$O/hash_sweep.json" 2> "$O/hash_sweep.err" || exit $?
for rep in 1 2; do
  for n in cur p0 p0r0 b16 p0w768 p0hw5; do
    L=$R/abtest/lib$n.so
    [ "$n" = cur ] && L=$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so
    TSDF_HIP_LIB=$L timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for vmm in 1 0; do
  TSDF_HASH_VMM=$vmm timeout -k 10 300 python -u tools/gpu/hash_pool_probe.py premapped >> "$O/pool.jsonl" 2>> "$O/pool.err" || exit $?
done
