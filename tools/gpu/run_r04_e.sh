# Round 4 call E: 16-frame launches.  b8 = the in-tree build (8 frames per launch everywhere),
# b16 = 16 everywhere, b16f8 = 16 for shards, 8 for whole volumes.  The driver-window probe for
# whole volumes (dense + hash), then rank 0 of eighth and quarter shards (dense, hash).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_e"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
for rep in 1 2; do
  for n in b8 b16 b16f8; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for rep in 1 2; do
  for n in b8 b16; do
    echo "$n s8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 48 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    echo "$n s4 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --only 4:0 --steps 1000 --warmup 48 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
