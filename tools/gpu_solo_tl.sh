#!/bin/bash
# CDR_PAR_SOLO sweep around the best point, then the C4/C5 kernel timelines at SOLO_TL
set -o pipefail
out=gpurun_out/${1:-solotl}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for so in ${SOLO_LIST:-2 4 8}; do
    CDR_PAR_SOLO=$so timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 cadence_amd/libcdr.so > $out/c${c}_$so.log 2>&1 || { tail -5 $out/c${c}_$so.log; exit 1; }
    echo "C$c solo=$so $(grep median_ms $out/c${c}_$so.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_ms"], d["checksum"])')"
  done
  CDR_PAR_SOLO=${SOLO_TL:-4} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tl/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/tl/c${c}_q4.log 2>&1 || exit 1
done
python3 tools/kernel_timeline.py $out/tl > $out/timeline.txt 2>&1; cat $out/timeline.txt
