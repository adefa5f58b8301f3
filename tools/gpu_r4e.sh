#!/bin/bash
# tools/gpu_r4d.sh (task + parity tests, the long-history A/B), then C3-C5 step times
# (1M workflows each, no oracle leg) — usage: tools/gpu_r4e.sh <tag>
set -o pipefail
tag=${1:-r4e}
tools/gpu_r4d.sh $tag ${tag}_lab || exit $?
out=gpurun_out/$tag
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $out/c$c.json 2> $out/c$c.log || exit 1
done
