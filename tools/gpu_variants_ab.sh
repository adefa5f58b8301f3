#!/bin/bash
# A/B of libcdr variants (variants/*.so, tools/build_variants.sh) against the main build on 1M-workflow configs
set -o pipefail
out=gpurun_out/${1:-vab}; shift; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  timeout -k 10 400 python3 tools/perf.py --config $c --rounds ${ROUNDS:-3} --reps 3 cadence_amd/libcdr.so "$@" > $out/c$c.json 2>$out/c$c.err || exit 1
  cat $out/c$c.json
done
