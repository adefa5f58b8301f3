#!/bin/bash
# A/B step times: libcdr.so against variants/libcdr_<name>.so, alternating (A B A B) per
# config, 1M workflows, no oracle leg.  usage: tools/gpu_ab.sh <tag> <name> <configs...>
set -o pipefail
tag=$1; name=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for c in "$@"; do
  for r in 1 2; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh > $out/c${c}_A$r.json 2> $out/c${c}_A$r.log || exit 1
    CDR_LIB=variants/libcdr_$name.so timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh > $out/c${c}_B$r.json 2> $out/c${c}_B$r.log || exit 1
  done
done
