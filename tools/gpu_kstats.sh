#!/bin/bash
# rocprofv3 kernel stats of the C3-C5 steps (1M workflows): gpurun_out/<tag>/c<N>/
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c$c -o run -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh > $out/c$c.json 2> $out/c$c.log || exit 1
done
