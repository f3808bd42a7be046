# A/B of library builds on the bench (dense + hash, no side legs): the in-tree library ("base")
# and abtest/lib<name>.so for each name given, interleaved twice.
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for name in base "$@"; do
    if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-mesh --no-ingest --no-dropin > gpurun_out/ab/$name.$rep.json 2> gpurun_out/ab/$name.$rep.err || exit $?
    echo "$name $rep $(grep -h 'dense:' gpurun_out/ab/$name.$rep.err | sed 's/.*-> //;s/ frames.*//') $(grep -h 'hash:' gpurun_out/ab/$name.$rep.err | sed 's/.*hash: //;s/ frames.*//')" >> gpurun_out/ab/summary.txt
  done
done
cat gpurun_out/ab/summary.txt
