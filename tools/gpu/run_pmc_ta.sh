# Memory-pipeline counters of the dense integrate (TA/TD/TCP gather throughput vs VALU), three
# separate rocprofv3 --pmc passes, kernel-trace only.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/pmc_ta"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmc_$name -o pmc -- python "$R/bench.py" --steps 400 --warmup 40 --no-hash --no-cpu --no-profile --no-ingest --no-mesh > "$O/$name.json" 2> "$O/$name.err" || return $?
  f=$(find /tmp/pmc_$name -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "k_integrate|Counter_Name" "$f" > "$O/$name.csv"
  return 0
}
pass a TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE &&
pass b TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES &&
pass c TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES TD_TD_BUSY &&
pass d SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU
