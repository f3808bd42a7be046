# Round 4 final call, on the committed in-tree library (no rebuild): the GPU tests and smoke
# (tools/gpu/run_tests.sh), the driver's bench command, then the round profile
# (tools/gpu/run_round_prof.sh: rocprofv3 stats of the driver's command, PMC traffic and SQ passes).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r04_final
bash tools/gpu/run_tests.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_final/bench_driver_args.json 2> gpurun_out/r04_final/bench.err || exit $?
bash tools/gpu/run_round_prof.sh
rc=$?
[ $rc -eq 0 ] || exit $rc
# (then, exploratory: call M's A/B of the entry-word read-modify-write and the hash protocol counts)
O="$R/gpurun_out/r04_m"
mkdir -p "$O"
TSDF_HIP_LIB=$R/abtest/libhdiag.so timeout -k 10 200 python -u tools/gpu/hash_diag.py > "$O/hash_diag.jsonl" 2> "$O/hash_diag.err" || exit $?
for n in cur occ; do
  L=$R/abtest/lib$n.so; [ "$n" = cur ] && L=$R/union-thesis-slam_amd/tsdf_amd/lib/libtsdf_hip.so
  TSDF_HIP_LIB=$L timeout -k 10 300 python -u tools/gpu/ab_window.py 3 $n >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
done
