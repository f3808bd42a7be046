# Round profile evidence: rocprofv3 kernel stats of the bench (tools/gpu/run_stats_pass.sh), the
# FETCH/WRITE traffic passes and the SQ issue pass (tools/gpu/run_pmc_passes.sh);
# tools/summarize_profile.py [sq] <tag> turns gpurun_out/ into profiles/.
set -o pipefail
bash tools/gpu/run_stats_pass.sh || exit $?
bash tools/gpu/run_pmc_passes.sh
