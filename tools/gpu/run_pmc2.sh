set -o pipefail
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc2"
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/gpu/rcp_probe.hip -o /tmp/rcp_probe 2>/dev/null && timeout -k 10 60 /tmp/rcp_probe > "$R/gpurun_out/pmc2/rcp.txt" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/pmc_$i -o pmc -- python "$R/bench.py" --steps 400 --warmup 40 --no-hash --no-cpu --no-profile > "$R/gpurun_out/pmc2/bench_$i.json" 2> "$R/gpurun_out/pmc2/bench_$i.err" || exit $?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "tsdf|Counter_Name" "$f" > "$R/gpurun_out/pmc2/pass_$i.csv"
done
