# The hash sweep (with the reference's table sizes), the hash extraction times and the shard-8
# kernel profile (the rest of tools/gpu/measure.sh ran already).
set -o pipefail
export PYTHONPATH=$PWD/union-thesis-slam_amd
O=gpurun_out/measure
mkdir -p $O
timeout -k 10 300 python -u tools/hash_sweep.py > $O/hash_sweep.json 2> $O/hash_sweep.err || exit $?
timeout -k 10 300 python -u tools/gpu/hash_extract_time.py > $O/hash_extract.json 2> $O/hash_extract.err || exit $?
bash tools/gpu/run_prof_shard8.sh
