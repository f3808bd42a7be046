# Per-kernel times of the in-line path (TSDF_PIPELINE=0): full-volume dense bench and rank 0 of the
# 8-way shard, rocprofv3 --kernel-trace --stats.   [out subdir, default inl; TSDF_HIP_LIB selects a variant]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-inl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
TSDF_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/q1 -o run --output-format csv -- python "$R/bench.py" --steps 1000 --warmup 50 --no-hash --no-cpu --no-mesh --no-ingest > $O/full.json 2> $O/full.err || exit $?
find /tmp/q1 -name "*kernel_stats.csv" -exec cp {} $O/full_stats.csv \;
TSDF_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/q2 -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 1000 --warmup 50 > $O/s8.json 2> $O/s8.err || exit $?
find /tmp/q2 -name "*kernel_stats.csv" -exec cp {} $O/s8_stats.csv \;
