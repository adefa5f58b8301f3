#!/bin/bash
set -o pipefail
out=gpurun_out/cuexp; mkdir -p $out
for k in 0 16 8 4; do
  for c in 4 5; do
    CDR_WAVE_CUS=$k timeout -k 10 200 python3 tools/perf.py --config $c --wfs 1000000 --rounds 2 --reps 2 cadence_amd/libcdr.so > $out/c${c}_k$k.log 2>&1 || exit 1
    echo "c$c k$k $(grep -h '^{' $out/c${c}_k$k.log)"
  done
done
