# A/B of the host-ingest legs (pcie_inclusive, dropin) between the in-tree library ("base") and
# abtest/lib<name>.so, interleaved twice.
set -o pipefail
mkdir -p gpurun_out/abi
for rep in 1 2; do
  for name in base "$@"; do
    if [ $name = base ]; then unset TSDF_HIP_LIB; else export TSDF_HIP_LIB=$PWD/abtest/lib$name.so; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-mesh --no-lounge --no-hash > gpurun_out/abi/$name.$rep.json 2> gpurun_out/abi/$name.$rep.err || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/abi/$name.$rep.json').read().strip().splitlines()[-1]); p=d['pcie_inclusive'] or {}; q=d['dropin'] or {}; print('$name $rep', d['value'], p.get('frames_per_s'), q.get('dense_frames_per_s'), q.get('hash_frames_per_s'), q.get('dense_undeferred_frames_per_s'))" >> gpurun_out/abi/summary.txt
  done
done
cat gpurun_out/abi/summary.txt
