# Round 4 A/B 1 at the driver's window (tools/gpu/ab_window.py): r4a (round-3 kernels with the
# round-4 host changes), r4b (hash z-halves claim at the end, scalar touched masks), r4c (r4b + the
# overlapped report-based settle of deferred hash batches), hotd (dense hot path only: an
# experiment, not correct in general); then the per-frame drop-in rates of r4a and r4c.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_ab1"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
for rep in 1 2; do
  for n in r4a r4b r4c r4d hotd lazy expect; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 5 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for n in r4a r4d; do
  echo "$n $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 2>> $O/dropin.err)" >> "$O/dropin.txt" || exit $?
done
# 16-frame batches (a build option): the whole bench at the driver window, and rank 0 of the
# eighth dense shard / eighth hash shard against the 8-frame build (r4c)
TSDF_HIP_LIB=$R/abtest/libb16.so timeout -k 10 300 python -u tools/gpu/ab_window.py 3 b16 >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
for rep in 1 2; do
  for n in r4d b16; do
    echo "$n s8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 48 2>> $O/s8.err)" >> "$O/shard8.txt" || exit $?
    echo "$n h8 $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s8.err)" >> "$O/shard8.txt" || exit $?
  done
done
