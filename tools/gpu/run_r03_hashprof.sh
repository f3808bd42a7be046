# Hash shards: kernel time of the fused hash launch at 1 and 8 ranks (rocprofv3 stats) against the
# wall-clock rate scaling_sim reports; then the measurement leftovers (load sweep, extraction).
set -o pipefail
export PYTHONPATH=$PWD/union-thesis-slam_amd
O=gpurun_out/hp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1 -o run -- python3 tools/scaling_sim.py --hash --worlds 1 --steps 400 > $O/h1.json 2> $O/h1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o run -- python3 tools/scaling_sim.py --hash --worlds 8 --steps 400 > $O/h8.json 2> $O/h8.err || exit $?
timeout -k 10 300 python -u tools/hash_sweep.py > $O/hash_sweep.json 2> $O/hash_sweep.err || exit $?
timeout -k 10 300 python -u tools/gpu/hash_extract_time.py > $O/hash_extract.json 2> $O/hash_extract.err || exit $?
