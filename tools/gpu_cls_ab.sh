#!/bin/bash
# A/B of the class-decomposed register-table kernel (k_replay_cls) on 1M-workflow C3-C5
set -o pipefail
out=gpurun_out/${1:-clsab}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python -u tools/perf.py --config $c --rounds 3 --reps 3 --ab-cls cadence_amd/libcdr.so > $out/c$c.json 2> $out/c$c.err || exit $?
  cat $out/c$c.json
done
