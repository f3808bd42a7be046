# Kernel times of one 8-way cyclic shard (rank 0 of 8) at 512^3: fused launches and the in-line
# kernels (TSDF_PIPELINE=0), rocprofv3 --kernel-trace --stats.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/shard8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in 1 0; do
  TSDF_PIPELINE=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ps8_$p -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 800 --warmup 48 > $O/p$p.json 2> $O/p$p.err || exit $?
  find /tmp/ps8_$p -name "*kernel_stats.csv" -exec cp {} $O/stats_p$p.csv \;
done
