#!/bin/bash
# kernel-class stream groupings at the box's 4 hardware queues (one process each:
# contexts in one process share the runtime's queues); class order of CDR_SIDE_GROUPS:
# wave, 12-activity, general, small-table, fast, 6-activity, PAR (7 = the caller's stream)
set -o pipefail
out=gpurun_out/${1:-grp}; mkdir -p $out
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"
for c in ${CONFIGS:-4 5 3}; do
  for g in ${GROUPS_LIST:-0555556 0075776 0675576 6005576 7575556 0123456}; do
    CDR_SIDE_GROUPS=$g timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/c${c}_$g.log 2>&1 || { tail -5 $out/c${c}_$g.log; exit 1; }
    echo "C$c $g $(grep median_ms $out/c${c}_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
  done
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/c${c}_q8.log 2>&1 || exit 1
  echo "C$c q8 $(grep median_ms $out/c${c}_q8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
done
