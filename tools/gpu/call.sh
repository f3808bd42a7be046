# One parameterised GPU call (replaces round 4's one-off run_r04_<x>.sh scripts):
#   bash tools/gpu/call.sh <out dir under gpurun_out/> <step> [<step> ...]
# Steps run in order, each under its own time limit; the call stops at the first failure.
#   tests              pytest -m gpu (in-tree library) + smoke
#   ab:<reps>:<a,b,..> driver-window A/B (tools/gpu/ab_window.py), libraries interleaved <reps>
#                      times; "base" = in-tree, anything else = abtest/lib<name>.so
#   bench[:<args>]     bench.py --gpus 1 --steps 20 --warmup 5 [args, '+'-separated]
#   sq[:<lib>]         one rocprofv3 --pmc SQ pass over the dense + hash bench legs
#   prof               the round profile (tools/gpu/run_round_prof.sh)
#   py:<script>[:args] python tools/gpu/<script> [args, '+'-separated]
#   pylib:<lib>:<script>[:args]  the same with TSDF_HIP_LIB=abtest/lib<lib>.so
set -o pipefail
O="gpurun_out/$1"
shift
mkdir -p "$O"
R=$(pwd)
lib() { case $1 in base|"") echo "";; *) echo "$R/abtest/lib$1.so";; esac; }
for step in "$@"; do
  echo "[call] $(date +%T) $step" | tee -a "$O/steps.log"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { echo "tests failed" >> "$O/steps.log"; exit 1; }
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
      ;;
    ab:*)
      IFS=: read -r _ reps names <<< "$step"
      IFS=, read -ra libs <<< "$names"
      for rep in $(seq 1 "$reps"); do
        for n in "${libs[@]}"; do
          TSDF_HIP_LIB=$(lib "$n") timeout -k 10 300 python tools/gpu/ab_window.py 3 "$n" >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit 1
        done
      done
      ;;
    bench*)
      args=${step#bench}; args=${args#:}; args=${args//+/ }
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 $args > "$O/bench.json" 2> "$O/bench.err" || exit 1
      ;;
    sq*)
      l=${step#sq}; l=${l#:}
      cd /tmp && export TMPDIR=/tmp
      TSDF_HIP_LIB=$(lib "$l") timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT \
        --kernel-trace --output-format csv -d /tmp/sq_$l -o pmc -- python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
        --no-cpu --no-profile --no-ingest --no-mesh --no-dropin --no-lounge > "$R/$O/sq_$l.json" 2> "$R/$O/sq_$l.err" || exit 1
      f=$(find /tmp/sq_$l -name "*counter_collection.csv" | head -1)
      [ -n "$f" ] && grep -E "k_fused|Counter_Name" "$f" > "$R/$O/sq_$l.csv"
      cd "$R"
      ;;
    prof)
      bash tools/gpu/run_round_prof.sh || exit 1
      ;;
    py:*)
      IFS=: read -r _ script args <<< "$step"
      timeout -k 10 600 python -u "tools/gpu/$script" ${args//+/ } > "$O/${script%.py}.out" 2> "$O/${script%.py}.err" || exit 1
      ;;
    pylib:*)
      IFS=: read -r _ l script args <<< "$step"
      TSDF_HIP_LIB=$(lib "$l") timeout -k 10 600 python -u "tools/gpu/$script" ${args//+/ } > "$O/${script%.py}_$l.out" \
        2> "$O/${script%.py}_$l.err" || exit 1
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[call] $(date +%T) done" | tee -a "$O/steps.log"
