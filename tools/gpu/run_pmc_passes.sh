# The two PMC traffic passes (FETCH_SIZE, WRITE_SIZE; --kernel-trace only beside --pmc) and the SQ
# pass, each the bench's dense and hash legs at the driver's window (--steps 20 --warmup 5): the
# counters of both integrate launches (k_fused, k_fused_hash) come from the same passes.
set -o pipefail
R=$(pwd)
O="$R/gpurun_out/profile"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
# RDREQ: the L2's memory-side read requests by size (TCC_EA0_RDREQ_{32B,64B,128B}): FETCH_SIZE tallies
# 128-B requests at 64 B on gfx950, so the read bytes are taken from the sizes themselves
# (tools/gpu/fetch_probe.hip checks the sum against known byte counts)
for pass in FETCH_SIZE WRITE_SIZE RDREQ; do
  i=$((i+1))
  counters=$pass
  [ $pass = RDREQ ] && counters="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d /tmp/pmc_$i -o pmc -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --no-profile --no-ingest --no-dropin --no-mesh --no-lounge > "$O/pmc_$pass.json" 2> "$O/pmc_$pass.err" || exit $?
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && grep -E "k_fused|Counter_Name" "$f" > "$O/pmc_$pass.csv"
done
cd "$R" && bash tools/gpu/run_pmc_sq.sh
