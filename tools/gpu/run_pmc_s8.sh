# SQ issue/wait breakdown of the dense integrate kernel on rank 0 of an 8-way cyclic shard.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/pmc_s8"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmc_s8 -o pmc -- python "$R/tools/scaling_sim.py" --only 8:0 --steps 400 --warmup 40 > "$O/s8.json" 2> "$O/s8.err" || exit $?
f=$(find /tmp/pmc_s8 -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && grep -E "k_integrate|k_cull|k_prep|Counter_Name" "$f" > "$O/pmc.csv"
