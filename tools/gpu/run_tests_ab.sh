# GPU tests + smoke, then the library A/B on the bench (tools/gpu/run_ab_bench.sh <names>).
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
bash tools/gpu/run_ab_bench.sh "$@"
