#!/bin/bash
# long-history routing sweep: configs 3-5 at 1M workflows under CDR_LONG="min,factor"
# values (one process each: the planner reads the override once); kernel stats per run
set -o pipefail
out=gpurun_out/${1:-long}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  for v in ${LONGS:-100000000,1 1024,2 512,1 2048,2}; do
    tag=c${c}_${v//,/_}
    CDR_LONG=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o run -- \
      python3 tools/perf.py --config $c --wfs 1000000 --rounds 2 --reps 2 cadence_amd/libcdr.so > $out/$tag.log 2>&1 || exit 1
    echo "$tag $(grep -h '^{' $out/$tag.log)"
  done
done
