# Generic A/B of library builds / environment settings on the bench and on rank 0 of eighth
# shards (dense columns and hash bucket ranges):
#   bash tools/gpu/ab.sh <out dir> <reps> <name>...
# name "base" = the in-tree library; "VAR=VAL[+VAR2=VAL2...]" = the in-tree library with those
# environment settings; anything else = abtest/lib<name>.so via TSDF_HIP_LIB.  Interleaved <reps> times.
# One summary line per run: name rep dense-fps hash-fps s8 dense-eighth-fps hash-eighth-fps.
set -o pipefail
O=$1; reps=$2; shift 2
mkdir -p $O
for rep in $(seq 1 $reps); do
  for name in "$@"; do
    unset TSDF_HIP_LIB
    envs=()
    case $name in
      base) ;;
      *=*) IFS='+' read -ra envs <<< "$name" ;;
      *) export TSDF_HIP_LIB=$PWD/abtest/lib$name.so ;;
    esac
    tag=${name//=/_}; tag=${tag//+/_}
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin > $O/$tag.$rep.json 2> $O/$tag.$rep.err || exit $?
    env "${envs[@]}" timeout -k 10 200 python tools/scaling_sim.py --only 8:0 --steps 1000 --warmup 50 > $O/s8_$tag.$rep.json 2> $O/s8_$tag.$rep.err || exit $?
    env "${envs[@]}" timeout -k 10 200 python tools/scaling_sim.py --hash --only 8:0 --steps 400 > $O/h8_$tag.$rep.json 2> $O/h8_$tag.$rep.err || exit $?
    echo "$tag $rep $(python -c "import json;d=json.load(open('$O/$tag.$rep.json'));print(d['value'],d['hash']['frames_per_s'])") s8 $(python -c "import json;print(json.load(open('$O/s8_$tag.$rep.json'))['fps'])") $(python -c "import json;print(json.load(open('$O/h8_$tag.$rep.json'))['hash8']['fps'])")" >> $O/summary.txt
  done
done
cat $O/summary.txt
