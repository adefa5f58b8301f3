#!/bin/bash
# Round 5, set B: the configs[4] conflict-resolution line at 1M with parity in the same run
# (canonical 48 + A[type] pricing, CPU baseline), and the multi-rank rehearsal of the
# --ndc-forks and --carry lines (ranks share the one GPU, counters reduced by gloo: the
# partition, per-rank parity and the reduction are what it shows, not scaling).
# usage: tools/gpu_r5b.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r5b}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 600 python -u bench.py --ndc-forks --steps 5 --warmup 1 > $out/ndc_forks_1m.json 2> $out/ndc_forks_1m.log || exit 1
export CDR_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --ndc-forks --gpus 2 --wfs 100000 --steps 3 --warmup 1 > $out/ndc_forks_n2.json 2> $out/ndc_forks_n2.log || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 \
  bench.py --carry --tasks --config 3 --gpus 2 --wfs 200000 --steps 3 --warmup 1 > $out/carry_tasks_c3_n2.json 2> $out/carry_tasks_c3_n2.log || exit 1
echo "r5b rc=0"
