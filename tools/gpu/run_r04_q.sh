# Round 4 call Q: progress priority for the dense integrate from 64 items per workgroup and for the
# hash from 16 (in-tree) against the previous defaults (prev: dense off, hash from 64) -- driver
# window and rank 0 of half / quarter / eighth shards; then the final-call steps on the in-tree
# build (tools/gpu/run_r04_final.sh without its exploratory tail) and the dense scaling prediction.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_q"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
lib() { if [ "$1" = cur ]; then echo "$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so"; else echo "$R/abtest/lib$1.so"; fi; }
for rep in 1 2; do
  for n in cur prev; do
    TSDF_HIP_LIB=$(lib $n) timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
    for w in 8:0 4:0 2:0; do
      echo "$n s$w $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --only $w --steps 1000 --warmup 48 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
    done
    echo "$n h8 $(TSDF_HIP_LIB=$(lib $n) timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 2>> $O/s.err)" >> "$O/shards.txt" || exit $?
  done
done
unset PYTHONPATH
cd "$R"
bash tools/gpu/run_tests.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONPATH="$R/union-thesis-slam_amd"
mkdir -p gpurun_out/r04_final
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_final/bench_driver_args.json 2> gpurun_out/r04_final/bench.err || exit $?
bash tools/gpu/run_round_prof.sh || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py > "$O/scaling_sim.json" 2> "$O/scaling_sim.err" || exit $?
