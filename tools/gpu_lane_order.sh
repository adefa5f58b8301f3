#!/bin/bash
# register-table lane order within a length class: by entity counts (default) vs footprint (CDR_LANE_ORDER_FOOTPRINT)
set -o pipefail
out=gpurun_out/${1:-lorder}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_counts.json 2>$out/c${c}_counts.err || exit 1
  CDR_LANE_ORDER_FOOTPRINT=1 timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_footprint.json 2>$out/c${c}_footprint.err || exit 1
  echo "C$c counts    $(head -1 $out/c${c}_counts.json) $(tail -1 $out/c${c}_counts.json | cut -c1-70)"
  echo "C$c footprint $(head -1 $out/c${c}_footprint.json) $(tail -1 $out/c${c}_footprint.json | cut -c1-70)"
done
