#!/bin/bash
# the whole GPU suite, then C3-C5 lines (full-size parity) and kernel timelines
set -o pipefail
tag=${1:-sb}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -60 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-stream-peak --no-refresh > $out/bench_c$c.log 2>&1 || { tail -30 $out/bench_c$c.log; exit 1; }
  grep -h '^{' $out/bench_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C$c', round(d['ms_per_step'],3), round(d['roofline']['frac'],4), d['parity']['mismatched_entries'])"
done
for c in ${TRACE:-3 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q4.log 2>&1 || exit 1
done
python3 tools/kernel_timeline.py $out > $out/timeline.txt 2>&1; cat $out/timeline.txt
