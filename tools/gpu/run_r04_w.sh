# Round 4 call W: later progress-priority steps for the hash on one GPU only (hlate,
# tools/patches/prio_levels_hash_late.py) against the final build: driver window (dense, hash) and
# the hash eighth shard, twice.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_w"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur hlate; do
    TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
