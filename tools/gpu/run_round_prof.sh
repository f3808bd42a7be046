# Round profile evidence: rocprofv3 kernel stats of the bench + FETCH/WRITE PMC passes
# (tools/gpu/run_profile.sh) + the SQ issue pass (tools/gpu/run_pmc_sq.sh).
set -o pipefail
bash tools/gpu/run_profile.sh || exit $?
bash tools/gpu/run_pmc_sq.sh
