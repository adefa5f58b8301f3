#!/bin/bash
# the longest PAR slices on CUs of their own (CDR_PAR_EXCL=K) vs shared CUs, separate processes
set -o pipefail
out=gpurun_out/${1:-excl}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for k in ${EXCLS:-0 4 8 16 32}; do
    CDR_PAR_EXCL=$k timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_$k -o run -- \
        python3 tools/perf.py --config $c --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$k.json 2>$out/c${c}_$k.err || exit 1
    echo "C$c excl=$k $(tail -1 $out/c${c}_$k.json | cut -c1-75)"
  done
done
