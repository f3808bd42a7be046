# PMC passes over a short dense-only bench (one counter group per rocprofv3 run, --kernel-trace
# only beside --pmc, as the MI355X guide prescribes).  Outputs the per-dispatch counter CSVs of
# the tsdf kernels into gpurun_out/pmc/.
set -o pipefail
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/pmc_$i -o pmc -- python "$R/bench.py" --steps 200 --warmup 20 --no-hash --no-cpu --no-profile > "$R/gpurun_out/pmc/bench_$i.json" 2> "$R/gpurun_out/pmc/bench_$i.err" || exit $?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "tsdf|Counter_Name|Dispatch_Id" "$f" | head -3000 > "$R/gpurun_out/pmc/pass_$i.csv"
  find /tmp/pmc_$i -type f | head -20 >> "$R/gpurun_out/pmc/files.txt"
done
