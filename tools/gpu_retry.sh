#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-rt}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  timeout -k 10 300 python3 -u tools/cls_retry.py --config $c > $out/c$c.log 2>&1 || { tail -20 $out/c$c.log; exit 1; }
  grep '^{' $out/c$c.log
done
