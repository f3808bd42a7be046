# Round 4 call P: the eighth-shard tail.  dp16 = progress priority for the dense integrate too,
# from 16 items per workgroup; pm16 = the hash's priority from 16 items (dense unchanged); dw512 =
# 512-thread dense workgroups (3 per CU).  Rank 0 of eighth shards (dense, hash) and the driver
# window, against the in-tree build.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_p"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur dp16 pm16 dw512; do
    echo "$n s8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 48 --kernel-time 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    echo "$n s4 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --only 4:0 --steps 1000 --warmup 48 --kernel-time 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --kernel-time --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
for n in cur dp16 pm16 dw512; do
  TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
done
