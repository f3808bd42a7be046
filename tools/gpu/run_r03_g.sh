# Round 3: GPU tests with the flat cull, then superbricks per cull workgroup (TSDF_CULL_G) again.
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
bash tools/gpu/ab.sh gpurun_out/g2 1 base TSDF_CULL_G=1 TSDF_CULL_G=2 TSDF_CULL_G=4
