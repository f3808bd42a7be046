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
  for n in r4a r4b r4c hotd; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 5 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for n in r4a r4c; do
  echo "$n $(TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 2>> $O/dropin.err)" >> "$O/dropin.txt" || exit $?
done
