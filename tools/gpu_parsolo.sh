#!/bin/bash
# CDR_PAR_SOLO sweep: the longest histories one per PAR slice (C4's tail: a 16-history PAR
# slice's W wave walks its histories round-robin, so the slice of the 16 longest sets the kernel's end)
set -o pipefail
out=gpurun_out/${1:-parsolo}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for so in ${SOLO_LIST:-0 4 16 64}; do
    CDR_PAR_SOLO=$so timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/c${c}_$so.log 2>&1 || { tail -5 $out/c${c}_$so.log; exit 1; }
    echo "C$c solo=$so $(grep median_ms $out/c${c}_$so.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
  done
done
