#!/bin/bash
# interleaved A/B of an env setting: ROUNDS passes over SETTINGS (each "VAR=val[,VAR=val]"),
# one perf.py process per (pass, setting), so box drift hits every setting alike
set -o pipefail
out=gpurun_out/${1:-ab}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for r in $(seq ${ROUNDS:-3}); do
    for s in ${SETTINGS:?}; do
      tag=c${c}_r${r}_${s//[=,]/_}
      env ${s//,/ } timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      echo "C$c r$r $s $(grep median_ms $out/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
    done
  done
done
