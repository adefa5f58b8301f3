#!/bin/bash
# Round 5, set L: kernel timelines of the C3 / C4 / C5 steps (rocprofv3 kernel trace over
# tools/perf.py, 1M workflows) — which class kernel ends each step.
set -o pipefail
out=gpurun_out/${1:-r5l}; mkdir -p $out
export TMPDIR=/tmp
for c in 3 4 5; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $out/c$c -o run -- python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c$c.log 2>&1 || exit 1
done
echo done
