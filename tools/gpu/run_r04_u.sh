# Round 4 call U: progress-priority steps (tools/patches/prio_levels.py): pl_late 12,14,15 and
# pl_early 4,8,12 sixteenths against the final build's 8,13,15 -- driver window, eighth shards.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_u"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur pl_late pl_early; do
    TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
