#!/bin/bash
# rocprofv3 kernel traces of C4 and C5 replays (timeline per kernel class)
set -o pipefail
out=gpurun_out/${1:-tr45}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$c -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c$c.log 2>&1 || exit 1
done
