#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-nolong}; mkdir -p $out
export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$c -o run -- \
    python3 tools/perf.py --config $c --rounds 1 --reps 3 --no-long cadence_amd/libcdr.so > $out/c$c.json 2>$out/c$c.err || exit 1
  cat $out/c$c.json
done
