#!/bin/bash
# PAR slice budget (CDR_PAR_MAX, slices) x PAR threshold factor (CDR_LONG's 4th field):
# with the wave class empty, the PAR kernel sets C4's critical path
set -o pipefail
out=gpurun_out/${1:-partune}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  for pm in ${PARMAX_LIST:-128 96 64 160}; do
    for pf in ${PARF_LIST:-1 2}; do
      CDR_PAR_MAX=$pm CDR_LONG=1024,2,2,$pf timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/c${c}_${pm}_$pf.log 2>&1 || { tail -5 $out/c${c}_${pm}_$pf.log; exit 1; }
      echo "C$c max=$pm f=$pf $(grep median_ms $out/c${c}_${pm}_$pf.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
    done
  done
done
