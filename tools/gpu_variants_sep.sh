#!/bin/bash
# A/B of libcdr builds in SEPARATE processes (one context per process: each gets the HIP
# hardware queues its kernel-class streams need; two contexts in one process share them)
set -o pipefail
out=gpurun_out/${1:-vsep}; shift; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  for rep in 1 2; do
    for lib in cadence_amd/libcdr.so "$@"; do
      n=$(basename $lib .so)
      timeout -k 10 300 python3 tools/perf.py --config $c --rounds ${ROUNDS:-3} --reps 3 $lib > $out/c${c}_${n}_$rep.json 2>$out/c${c}_${n}_$rep.err || exit 1
      echo "C$c $n $rep $(tail -1 $out/c${c}_${n}_$rep.json | cut -c1-75)"
    done
  done
done
