#!/bin/bash
# kernel-class launch orders (CDR_LAUNCH_ORDER) on C3-C5
set -o pipefail
out=gpurun_out/${1:-order}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  for o in ${ORDERS:-6012345 6501234 5601234 6153024}; do
    CDR_LAUNCH_ORDER=$o timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$o.json 2>$out/c${c}_$o.err || exit 1
    echo "C$c $o $(tail -1 $out/c${c}_$o.json | cut -c1-80)"
  done
done
