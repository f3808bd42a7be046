# Launch gaps of the fused dense launch: rocprofv3 kernel trace of rank 0 of 8 and of one GPU
# (scaling_sim --only), summarised on the box by tools/launch_gaps.py into gpurun_out/gaps/
# (the trace CSVs stay in /tmp: they exceed what a call copies back).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/gaps
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gap_$w -o run --output-format csv -- python "$R/tools/scaling_sim.py" --only $w:0 --steps 400 --warmup 48 > $O/w$w.json 2> $O/w$w.err || exit $?
  python "$R/tools/launch_gaps.py" $(find /tmp/gap_$w -name "*kernel_trace.csv" | head -1) > $O/gaps_w$w.txt || exit $?
done
cat $O/gaps_w*.txt
