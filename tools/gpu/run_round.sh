# Round-end evidence in one call: GPU tests, smoke, default bench, scaling simulation, the
# multi-rank (gloo, shared GPU) rehearsal of the bench, then the rocprofv3 kernel-stats run and
# the two PMC passes (tools/gpu/run_profile.sh).
set -o pipefail
SCALE=1 bash tools/gpu/run_all.sh || exit $?
bash tools/gpu/run_multirank.sh || exit $?
bash tools/gpu/run_profile.sh
