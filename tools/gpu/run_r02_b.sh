# GPU tests + smoke + default bench (tools/gpu/run_all.sh), then the multi-rank rehearsal.
set -o pipefail
bash tools/gpu/run_all.sh || exit $?
bash tools/gpu/run_multirank.sh
