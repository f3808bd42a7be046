# Round 4 call J: strong-scaling prediction on the in-tree build (XCD-aware dealing, 768-thread
# hash workgroups): dense cyclic / slab shards, hash bucket-range shards at 512^3 and 1024^3; and
# workgroup timelines (diagnostic build abtest/libwgt.so) of dense shards and the hash.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_j"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
timeout -k 10 300 python -u tools/scaling_sim.py > "$O/scaling_sim.json" 2> "$O/scaling_sim.err" || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --kernel-time > "$O/scaling_sim_hash.json" 2> "$O/scaling_sim_hash.err" || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --kernel-time --extent 1024 --worlds 1,8 > "$O/scaling_sim_hash1024.json" 2> "$O/scaling_sim_hash1024.err" || exit $?
TSDF_HIP_LIB=$R/abtest/libwgt.so timeout -k 10 200 python -u tools/gpu/wg_times.py > "$O/wg_times.jsonl" 2> "$O/wg_times.err" || exit $?
TSDF_HIP_LIB=$R/abtest/libwgt.so timeout -k 10 200 python -u tools/gpu/wg_times_hash.py > "$O/wg_times_hash.jsonl" 2> "$O/wg_times_hash.err" || exit $?
