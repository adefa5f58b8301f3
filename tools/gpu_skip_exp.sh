#!/bin/bash
# timing-only experiment: the class kernels without their P loop / W loop (outputs wrong by
# construction; each library in its own process)
set -o pipefail
out=gpurun_out/${1:-skp}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4}; do
  for v in base skipp skipw; do
    timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 variants/libcdr_$v.so > $out/c${c}_$v.log 2>&1
    echo "C$c $v $(grep median_ms $out/c${c}_$v.log | cut -c1-90)"
  done
done
