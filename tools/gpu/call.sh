# One parameterised GPU call (replaces round 4's one-off run_r04_<x>.sh scripts):
#   bash tools/gpu/call.sh <out dir under gpurun_out/> <step> [<step> ...]
# Steps run in order, each under its own time limit; the call stops at the first failure.
#   tests              pytest -m gpu (in-tree library) + smoke
#   pytest:<args>      pytest -m gpu <args, '+'-separated> (a subset, e.g. pytest:tests/test_long_gpu.py+-k+config4)
#   pytestlib:<lib>:<args>  the same with TSDF_HIP_LIB=abtest/lib<lib>.so
#   testsenv:<VAR=VAL[+..]>  the whole -m gpu suite with that environment (no smoke)
#   ab:<reps>:<a,b,..> driver-window A/B (tools/gpu/ab_window.py), libraries interleaved <reps>
#                      times; "base" = in-tree, VAR=VAL[+..] = in-tree with that environment,
#                      anything else = abtest/lib<name>.so
#   abs:<reps>:<a,b,..> tools/gpu/ab.sh: the bench and rank 0 of eighth dense / hash shards, per build
#                      ("base", abtest/lib<name>.so, or VAR=VAL[+VAR2=VAL2] on the in-tree library)
#   bench[@tag][:<args>]  bench.py --gpus 1 --steps 20 --warmup 5 [args, '+'-separated] -> bench[_tag].json
#   gloo2[:<args>]     bench.py --gpus 2 --dist-backend gloo (two ranks on the one GPU) -> bench_gpus2_gloo.json
#   sq[:<lib>]         one rocprofv3 --pmc SQ pass over the dense + hash bench legs
#   prof               the round profile (tools/gpu/run_round_prof.sh)
#   py:<script>[:args] python tools/gpu/<script> [args, '+'-separated]
#   pylib:<lib>:<script>[:args]  the same with TSDF_HIP_LIB=abtest/lib<lib>.so
#   tool:<script>[:args]:<tag>  python tools/<script> [args], output to <dir>/<tag>.out
#   toolenv:<VAR=VAL[+..]>:<script>:<args>:<tag>  the same with that environment
#   bin:<path>         a prebuilt probe binary (tools/gpu/<name>), output to <dir>/<name>.out
#   kt:<script>[:args] the same under rocprofv3 --kernel-trace --stats (stats csv copied to <dir>)
#   pmcbin:<binary>:<c1+c2..>[:<c1+..>]  rocprofv3 --pmc passes over a prebuilt probe (csv to <dir>)
#   dropthreads:<t1+t2..>  per-frame drop-in rate per copy-pool size (tools/gpu/dropin_threads.sh)
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
    pytest:*)
      args=${step#pytest:}; args=${args//+/ }
      timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        $args > "$O/pytest_subset.log" 2>&1 || { echo "pytest subset failed" >> "$O/steps.log"; exit 1; }
      ;;
    testsenv:*)  # the whole GPU suite with VAR=VAL[+VAR2=VAL2] set (e.g. TSDF_TEXEL=1)
      IFS='+' read -ra envs <<< "${step#testsenv:}"
      env "${envs[@]}" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > "$O/gpu_tests_env.log" 2>&1 || { echo "tests (env) failed" >> "$O/steps.log"; exit 1; }
      ;;
    pytestlib:*)
      IFS=: read -r _ l args <<< "$step"; args=${args//+/ }
      TSDF_HIP_LIB=$(lib "$l") timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider $args > "$O/pytest_$l.log" 2>&1 || { echo "pytest $l failed" >> "$O/steps.log"; exit 1; }
      ;;
    ab:*)
      IFS=: read -r _ reps names <<< "$step"
      IFS=, read -ra libs <<< "$names"
      for rep in $(seq 1 "$reps"); do
        for n in "${libs[@]}"; do
          if [[ $n == *=* ]]; then  # VAR=VAL[+VAR2=VAL2] on the in-tree library
            IFS='+' read -ra envs <<< "$n"
            env "${envs[@]}" timeout -k 10 300 python tools/gpu/ab_window.py 3 "$n" >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit 1
          else
            TSDF_HIP_LIB=$(lib "$n") timeout -k 10 300 python tools/gpu/ab_window.py 3 "$n" >> "$O/ab.jsonl" 2>> "$O/ab.err" || exit 1
          fi
        done
      done
      ;;
    abs:*)
      IFS=: read -r _ reps names <<< "$step"
      IFS=, read -ra libs <<< "$names"
      bash tools/gpu/ab.sh "$O/abs" "$reps" "${libs[@]}" > "$O/abs.out" 2>&1 || exit 1
      ;;
    gloo2*)
      # gloo2[:args]: the bench's multi-rank path, two ranks sharing the one GPU over gloo
      args=""; [[ $step == *:* ]] && args=${step#*:}; args=${args//+/ }
      timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 $args \
        > "$O/bench_gpus2_gloo.json" 2> "$O/bench_gpus2_gloo.err" || exit 1
      ;;
    bench*)
      # bench[@tag][:args]: output <dir>/bench[_tag].json
      head=${step%%:*}; tag=${head#bench}; tag=${tag#@}
      args=""; [[ $step == *:* ]] && args=${step#*:}; args=${args//+/ }
      out="$O/bench${tag:+_$tag}"
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 $args > "$out.json" 2> "$out.err" || exit 1
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
      TSDF_HIP_LIB=$(lib "$l") timeout -k 10 600 python -u "tools/gpu/$script" ${args//+/ } >> "$O/${script%.py}_$l.out" \
        2>> "$O/${script%.py}_$l.err" || exit 1
      ;;
    tool:*)
      IFS=: read -r _ script args tag <<< "$step"
      timeout -k 10 900 python -u "tools/$script" ${args//+/ } > "$O/$tag.out" 2> "$O/$tag.err" || exit 1
      ;;
    toolenv:*)  # toolenv:VAR=VAL[+VAR2=VAL2]:<script>:<args>:<tag> -- tool: with that environment
      IFS=: read -r _ envspec script args tag <<< "$step"
      IFS='+' read -ra envs <<< "$envspec"
      env "${envs[@]}" timeout -k 10 900 python -u "tools/$script" ${args//+/ } > "$O/$tag.out" 2> "$O/$tag.err" || exit 1
      ;;
    bin:*)
      b=${step#bin:}
      timeout -k 10 120 "./$b" > "$O/$(basename "$b").out" 2>&1 || exit 1
      ;;
    dropthreads:*)
      # dropthreads:<t1+t2+..>  the per-frame drop-in rate for each copy-pool size (dropin_threads.sh)
      ts=${step#dropthreads:}
      bash tools/gpu/dropin_threads.sh "$O/dropin_threads.jsonl" ${ts//+/ } 2> "$O/dropin_threads.err" || exit 1
      ;;
    pmcbin:*)
      # pmcbin:<binary>:<pass>[:<pass>..], each pass '+'-separated counters: one rocprofv3 --pmc run of
      # the prebuilt probe per pass (kernel-trace only beside the counters), csv into <dir>
      IFS=: read -r _ b passes <<< "$step"
      IFS=: read -ra plist <<< "$passes"
      k=0
      for pc in "${plist[@]}"; do
        k=$((k+1))
        cd /tmp && export TMPDIR=/tmp
        timeout -s KILL 120 rocprofv3 --pmc ${pc//+/ } --kernel-trace --output-format csv -d /tmp/pmcbin_$k -o p -- \
          "$R/$b" > "$R/$O/$(basename "$b")_pass$k.out" 2>&1 || exit 1
        f=$(find /tmp/pmcbin_$k -name "*counter_collection.csv" | head -1)
        [ -n "$f" ] && cp "$f" "$R/$O/$(basename "$b")_pass$k.csv"
        cd "$R"
      done
      ;;
    kt:*)
      IFS=: read -r _ script args <<< "$step"
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_${script%.py} -o kt -- \
        python -u "$R/tools/gpu/$script" ${args//+/ } > "$R/$O/kt_${script%.py}.out" 2> "$R/$O/kt_${script%.py}.err" || exit 1
      f=$(find /tmp/kt_${script%.py} -name "*kernel_stats.csv" | head -1)
      [ -n "$f" ] && cp "$f" "$R/$O/kt_${script%.py}_kernel_stats.csv"
      f=$(find /tmp/kt_${script%.py} -name "*kernel_trace.csv" | head -1)
      [ -n "$f" ] && cp "$f" "$R/$O/kt_${script%.py}_kernel_trace.csv"
      cd "$R"
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[call] $(date +%T) done" | tee -a "$O/steps.log"
