# Round 4 A/B 1 at the driver's window (tools/gpu/ab_window.py): r4a (round-3 kernels with the
# round-4 host changes), r4e (hash: cull lookup, missing blocks from the fresh state, claim at the
# end), r4f (r4e + volume / pool / table fields read through opaque kernarg pointers: no SGPR
# spills to VGPR lanes, no hash scratch), w8 / w8s (r4f at 8 waves/SIMD, 1024- / 512-thread
# workgroups); the per-frame drop-in rates of r4a and r4f; rank 0 of eighth shards for r4f, w8
# and b16 (16-frame batches).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_ab1"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
for rep in 1 2; do
  for n in r4a r4e r4f w8 w8s; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 5 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for n in r4a r4f; do
  echo "$n $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 2>> $O/dropin.err)" >> "$O/dropin.txt" || exit $?
done
for rep in 1 2; do
  for n in r4f w8 b16; do
    echo "$n s8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 48 2>> $O/s8.err)" >> "$O/shard8.txt" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s8.err)" >> "$O/shard8.txt" || exit $?
  done
done
