# Round 4 call V: PMC counters of the hash launch in the bench's hash leg (fresh table: 20 timed
# launches that insert 72.5k blocks, then the same window again without inserts), each counter set
# in its own rocprofv3 --pmc pass (kernel-trace only beside it): HBM bytes and SQ issue / wait, to
# see where the inserting window's extra time goes.  tools/hash_pmc_summary.py reads the result.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/r04_v"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu --no-profile --no-ingest --no-mesh --no-dropin --no-lounge"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d /tmp/pmc_v$i -o pmc -- python "$R/bench.py" $ARGS > "$O/pass$i.json" 2> "$O/pass$i.err" || exit $?
  f=$(find /tmp/pmc_v$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "k_fused_hash|Counter_Name" "$f" > "$O/pass$i.csv"
done
exit 0
