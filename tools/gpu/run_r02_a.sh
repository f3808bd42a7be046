# GPU tests, hash load-factor sweep, in-line-path kernel stats at the 1024^3 extent (k_cull cost),
# scaling simulation.
set -o pipefail
mkdir -p gpurun_out/r02a
R=$(pwd)
O=$R/gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python tools/hash_sweep.py > $O/hash_sweep.json 2> $O/hash_sweep.err || exit $?
timeout -k 10 600 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/scaling_sim.err || exit $?
cd /tmp && export TMPDIR=/tmp
TSDF_PIPELINE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_inl -o run --output-format csv -- python "$R/tools/hash_sweep.py" --loads 0.5 --frames 200 > $O/inline_sweep.json 2> $O/inline_sweep.err || exit $?
find /tmp/prof_inl -name "*kernel_stats.csv" -exec cp {} $O/inline_kernel_stats.csv \;
