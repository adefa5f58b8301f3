#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: N ranks through
# torch.distributed.run sharing the device, counters reduced with gloo on the host
# (CDR_BENCH_BACKEND=gloo; the driver's 8-GPU runs use RCCL).  Shard assignment,
# per-rank batches, the barrier / max-over-ranks timing and the per-rank parity run as
# on a node.  usage: tools/gpu_multirank.sh <tag>
set -o pipefail
out=gpurun_out/${1:-mr}; mkdir -p $out
export CDR_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --wfs 300000 --steps 5 --warmup 2 --no-cpu-baseline --no-refresh --no-stream-peak > $out/c2_n2.json 2> $out/c2_n2.log || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 4 --config 4 --wfs 100000 --steps 3 --warmup 1 --no-cpu-baseline --no-refresh --no-stream-peak > $out/c4_n4.json 2> $out/c4_n4.log || exit 1
