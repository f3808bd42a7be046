# Round 4 call R, on the final in-tree build (0994d6651dd66c38): the driver's bench command three more times (run-to-
# run spread) and the scaling prediction (dense, hash 512^3, hash 1024^3) of the same build.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_r"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu >> "$O/bench_repeats.jsonl" 2>> "$O/bench.err" || exit $?
done
timeout -k 10 300 python -u tools/scaling_sim.py > "$O/scaling_sim.json" 2> "$O/scaling_sim.err" || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --kernel-time > "$O/scaling_sim_hash.json" 2> "$O/scaling_sim_hash.err" || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --kernel-time --extent 1024 --worlds 1,8 > "$O/scaling_sim_hash1024.json" 2> "$O/scaling_sim_hash1024.err" || exit $?
