# SQ issue/wait breakdown of the integrate launches (k_fused, k_fused_hash) at the driver's window
# (one rocprofv3 --pmc pass over the dense and hash legs, kernel-trace only).
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/pmc_sq"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmc_sq -o pmc -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --no-profile --no-ingest --no-mesh --no-dropin --no-lounge > "$O/bench.json" 2> "$O/bench.err" || exit $?
f=$(find /tmp/pmc_sq -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && grep -E "k_fused|k_integrate|Counter_Name" "$f" > "$O/pmc_sq.csv"
exit 0
