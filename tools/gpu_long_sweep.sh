#!/bin/bash
# long-history threshold sweep (CDR_LONG="min,factor,reg2 divisor"), separate processes,
# each under a kernel trace so the per-kernel end times can be read
set -o pipefail
out=gpurun_out/${1:-long}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for v in ${LONGS:-1024,2,2 1024,1,2 512,1,2 2048,4,2}; do for pm in ${PARMAX:-256}; do
    t=${v//,/_}_$pm
    CDR_PAR_MAX=$pm CDR_LONG=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_$t -o run -- \
        python3 tools/perf.py --config $c --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$t.json 2>$out/c${c}_$t.err || exit 1
    echo "C$c long=$v parmax=$pm $(tail -1 $out/c${c}_$t.json | cut -c1-75)"
  done; done
done
