# Round 3: per-role workgroup timeline of the fused dense launch (abtest/libwgt.so), then
# bench / eighth-shard A/B of the in-tree library against the ungated hash priority.
set -o pipefail
TSDF_HIP_LIB=$PWD/abtest/libwgt.so timeout -k 10 240 python -u tools/gpu/wg_times.py > gpurun_out/wg_roles.txt 2>&1 || exit $?
bash tools/gpu/ab.sh gpurun_out/prio3 2 base nohp
