#!/bin/bash
# C3-C5 bench lines (full-size parity) + kernel timelines at the box's queue setting
set -o pipefail
tag=${1:-c345}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-stream-peak --no-refresh ${BENCH_ARGS} > $out/bench_c$c.log 2>&1 || { tail -30 $out/bench_c$c.log; exit 1; }
  grep -h '^{' $out/bench_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C$c', round(d['ms_per_step'],3), round(d['roofline']['frac'],4), d['parity'] and d['parity']['mismatched_entries'])"
done
for c in ${TRACE:-3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q4.log 2>&1 || exit 1
done
python3 tools/kernel_timeline.py $out > $out/timeline.txt 2>&1; cat $out/timeline.txt
