#!/bin/bash
# Step time of a config under each of several environment settings (1M workflows, no oracle
# leg, two passes in alternating order).  usage: tools/gpu_sweep.sh <tag> <config> VAR=v1 VAR=v2 ...
set -o pipefail
tag=$1; c=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in 1 2; do
  for e in "$@"; do
    n=$(echo "$e" | tr '=,' '__')
    env $e timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh $BENCH_ARGS > $out/c${c}_${n}_$r.json 2> $out/c${c}_${n}_$r.log || exit 1
  done
done
