# Rehearsal of the multi-rank bench path on a one-GPU box: 2 and 4 ranks share the GPU over gloo
# (the driver's 8-GPU runs use one GPU per rank over RCCL).  Checks that every rank runs, the
# max-over-ranks timing and the sums work, and rank 0 prints one JSON line.
set -o pipefail
mkdir -p gpurun_out/mr
for n in 2 4; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 50 --warmup 5 --dist-backend gloo --no-cpu \
    > gpurun_out/mr/n$n.json 2> gpurun_out/mr/n$n.err || exit $?
done
