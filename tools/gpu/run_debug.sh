set -o pipefail
mkdir -p gpurun_out
for m in 1 2 3; do
  echo "=== TSDF_DEBUG=$m" >> gpurun_out/debug_hash.log
  TSDF_DEBUG=$m timeout -k 10 300 python tools/gpu/debug_hash.py >> gpurun_out/debug_hash.log 2>&1 || exit 1
done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude -Iunion-thesis-slam_amd/csrc --save-temps -c union-thesis-slam_amd/csrc/tsdf_hash.hip -o /tmp/h.o 2>/dev/null; cp tsdf_hash-hip-amdgcn-amd-amdhsa-gfx950.s gpurun_out/ 2>/dev/null; true
