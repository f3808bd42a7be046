# Hash shard scaling after the owned-brick cull: 512^3 (1/2/4/8) and 1024^3 (1, 8).
set -o pipefail
export PYTHONPATH=$PWD/union-thesis-slam_amd
O=gpurun_out/measure3
mkdir -p $O
timeout -k 10 300 python -u tools/scaling_sim.py --hash --steps 400 > $O/scaling_sim_hash.json 2> $O/scaling_sim_hash.err || exit $?
timeout -k 10 400 python -u tools/scaling_sim.py --hash --extent 1024 --worlds 1,8 --steps 400 > $O/hash_shard8_1024.json 2> $O/hash_shard8_1024.err || exit $?
