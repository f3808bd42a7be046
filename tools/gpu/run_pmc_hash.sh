# SQ issue counters of the hash launch (k_fused_hash) and of the dense launch at NZ = 8 / 4 waves
# per SIMD (abtest/libw4.so, TSDF_DENSE_NZ=8): where the hash's extra time goes.
# Build the variant first: tools/build_variant.sh w4 "-DTSDF_DENSE_WAVES=4"
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/pmc_hash"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d /tmp/pmc_h -o pmc -- python "$R/bench.py" --steps 50 --warmup 5 --no-cpu --no-profile --no-ingest --no-mesh --no-dropin --no-lounge > "$O/hash.json" 2> "$O/hash.err" || exit $?
f=$(find /tmp/pmc_h -name "*counter_collection.csv" | head -1); grep -E "k_fused|Counter_Name" "$f" > "$O/hash.csv"
TSDF_HIP_LIB=$R/abtest/libw4.so TSDF_DENSE_NZ=8 timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d /tmp/pmc_d8 -o pmc -- python "$R/bench.py" --steps 50 --warmup 5 --no-hash --no-cpu --no-profile --no-ingest --no-mesh --no-dropin --no-lounge > "$O/d8.json" 2> "$O/d8.err" || exit $?
f=$(find /tmp/pmc_d8 -name "*counter_collection.csv" | head -1); grep -E "k_fused|Counter_Name" "$f" > "$O/d8.csv"
