# Round 4 call T: cull workgroup size (TSDF_CULL_G superbricks per workgroup, run-time switch) on the
# final build, now that progress priority keeps every integrate workgroup busy until the launch's
# last ~100 us and the cull / prep stages run in its tail; driver window, twice each.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_t"
mkdir -p "$O"
export PYTHONPATH="$R/union-thesis-slam_amd"
for rep in 1 2; do
  for g in 3 1 2 4; do
    TSDF_CULL_G=$g timeout -k 10 300 python -u tools/gpu/ab_window.py 3 g$g >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit $?
  done
done
