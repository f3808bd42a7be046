# Round 4 call G: the driver's bench command on the in-tree build (r4l: 16-frame launches, next-
# item prefetch, per-item volume locals, deferred batches of 8), the driver-window A/B against
# b16 (16-frame launches without the prefetch / locals), the per-frame drop-in rates with deferred
# batches of 8 and 16 frames, and the load-factor sweep.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_g"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || exit $?
for rep in 1 2; do
  for n in b16 r4l; do
    TSDF_HIP_LIB=$R/abtest/lib$n.so timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
for df in 8 16; do
  echo "defer_frames=$df $(TSDF_DEFER_FRAMES=$df timeout -k 10 300 python -u tools/gpu/dropin_rate.py 256 5 2>> $O/dropin.err | tail -1)" >> "$O/dropin.txt" || exit $?
done
timeout -k 10 500 python -u tools/hash_sweep.py > "$O/hash_sweep.json" 2> "$O/hash_sweep.err" || exit $?
