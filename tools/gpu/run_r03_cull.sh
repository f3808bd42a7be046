# Round 3: cull workgroups of G superbricks by volume size: GPU tests on the in-tree library, the
# per-role timeline (abtest/libwgt.so), the bench / eighth-shard A/B against G = 1, quarter and
# half shards at G = 1 / 2 / 3, and the launch gaps.
set -o pipefail
bash tools/gpu/run_tests.sh || exit $?
TSDF_HIP_LIB=$PWD/abtest/libwgt.so timeout -k 10 240 python -u tools/gpu/wg_times.py > gpurun_out/wg_roles_rule.txt 2>&1 || exit $?
bash tools/gpu/ab.sh gpurun_out/cull2 2 base TSDF_CULL_G=1 || exit $?
for rep in 1 2; do for g in 1 2 3; do for w in 2 4; do
  TSDF_CULL_G=$g timeout -k 10 200 python tools/scaling_sim.py --only $w:0 --steps 1000 --warmup 50 > gpurun_out/cull2/w${w}_g$g.$rep.json 2>/dev/null || exit $?
  echo "w$w g$g $rep $(python -c "import json;print(json.load(open('gpurun_out/cull2/w${w}_g$g.$rep.json'))['fps'])")" >> gpurun_out/cull2/shards.txt
done; done; done
cat gpurun_out/cull2/shards.txt
bash tools/gpu/run_gaps.sh
