#!/bin/bash
# stream-priority masks (CDR_STREAM_PRIO, bit i = side stream i at high priority) on C3-C5
set -o pipefail
out=gpurun_out/${1:-sprio}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  for m in ${MASKS:-0x47 0x7f 0x00 0x67 0x40}; do
    CDR_STREAM_PRIO=$m timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$m.json 2>$out/c${c}_$m.err || exit 1
    echo "C$c $m $(tail -1 $out/c${c}_$m.json | cut -c1-80)"
  done
done
