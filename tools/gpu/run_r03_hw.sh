# Round 3: the fused hash launch at 5 waves / SIMD (abtest/libhw5.so: fewer spills) and with
# 768-thread workgroups (abtest/libhwg1k.so) against the in-tree library.
set -o pipefail
bash tools/gpu/ab.sh gpurun_out/hw 2 base hw5 hwg1k
