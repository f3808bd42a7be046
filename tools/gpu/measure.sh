# Round 3 measurements on one GPU: strong-scaling simulation (dense columns and hash bucket
# ranges), config[4]'s per-rank hash shard, the load-factor sweep on the fused launch, and the
# on-device hash extraction.  Outputs under gpurun_out/measure/.
set -o pipefail
export PYTHONPATH=$PWD/union-thesis-slam_amd
O=gpurun_out/measure
mkdir -p $O
timeout -k 10 400 python -u tools/scaling_sim.py > $O/scaling_sim.json 2> $O/scaling_sim.err || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --steps 400 > $O/scaling_sim_hash.json 2> $O/scaling_sim_hash.err || exit $?
timeout -k 10 300 python -u tools/scaling_sim.py --hash --extent 1024 --worlds 1,8 --steps 400 > $O/hash_shard8_1024.json 2> $O/hash_shard8_1024.err || exit $?
timeout -k 10 300 python -u tools/hash_sweep.py > $O/hash_sweep.json 2> $O/hash_sweep.err || exit $?
timeout -k 10 300 python -u tools/gpu/hash_extract_time.py > $O/hash_extract.json 2> $O/hash_extract.err || exit $?
