# Round 3 final evidence on the committed kernels: GPU tests + smoke, the default bench line,
# rocprofv3 kernel stats + PMC passes, the dense scaling simulation and shard-8 profile.

set -o pipefail
bash tools/gpu/run_evidence.sh || exit $?
export PYTHONPATH=$PWD/union-thesis-slam_amd
mkdir -p gpurun_out/measure4
timeout -k 10 400 python -u tools/scaling_sim.py > gpurun_out/measure4/scaling_sim.json 2> gpurun_out/measure4/scaling_sim.err || exit $?
bash tools/gpu/run_prof_shard8.sh || exit $?
