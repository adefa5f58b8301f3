#!/bin/bash
# A/B step times: libcdr.so against B, alternating (A B A B) per config, 1M workflows, no
# oracle leg.  B = a variant name (variants/libcdr_<name>.so) or env:VAR=value (libcdr.so
# under that environment).  Extra bench flags via BENCH_ARGS.
# (AENV=VAR=value: the A leg under that environment.)
# usage: tools/gpu_ab.sh <tag> <B> <configs...>
set -o pipefail
tag=$1; b=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
if [[ $b == env:* ]]; then benv=${b#env:}; else benv=CDR_LIB=variants/libcdr_$b.so; fi
for c in "$@"; do
  for r in 1 2; do
    env $AENV timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh $BENCH_ARGS > $out/c${c}_A$r.json 2> $out/c${c}_A$r.log || exit 1
    env $benv timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh $BENCH_ARGS > $out/c${c}_B$r.json 2> $out/c${c}_B$r.log || exit 1
  done
done
