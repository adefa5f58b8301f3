#!/bin/bash
# PAR slices: the longest K histories one per slice (CDR_PAR_SOLO=K) vs 16 per slice, separate processes
set -o pipefail
out=gpurun_out/${1:-solo}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for k in ${SOLOS:-0 16 64}; do
    CDR_PAR_SOLO=$k timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$k.json 2>$out/c${c}_$k.err || exit 1
    echo "C$c solo=$k $(tail -1 $out/c${c}_$k.json | cut -c1-75)"
  done
done
