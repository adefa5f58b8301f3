#!/bin/bash
# end-of-round set, part B: for C3-C5, PMC passes of the whole replay step -> traffic (same
# build), then the bench line (full-size parity, CPU baseline) that picks the traffic up
set -o pipefail
tag=${1:-r3f}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  bash tools/pmc.sh ${tag}c$c cadence_amd/libcdr.so --config $c > $out/pmc_c$c.log 2>&1 || { tail -20 $out/pmc_c$c.log; exit 1; }
  python3 tools/traffic.py ${tag}c$c C$c-1000000wf-sliced ${tag}_c$c k_replay k_tables > $out/traffic_c$c.log 2>&1 || { cat $out/traffic_c$c.log; exit 1; }
  cp profiles/traffic_C$c-1000000wf-sliced.json profiles/${tag}_c${c}_pmc.txt $out/
  timeout -k 10 400 python -u bench.py --config $c > $out/bench_c$c.log 2>&1 || { tail -30 $out/bench_c$c.log; exit 1; }
  grep -h '^{' $out/bench_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C$c', round(d['ms_per_step'],3), round(r['frac'],4), r['traffic'], d['parity']['mismatched_entries'])"
done
