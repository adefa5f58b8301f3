#!/bin/bash
# round 3: GPU suite, then C3-C5 lines with the host-packed class blocks under both stream
# layouts (3 grouped side streams at HIP's default 4 hardware queues; 7 at 8 queues)
set -o pipefail
tag=${1:-r3a}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-stream-peak --no-refresh > $out/bench_c${c}_q4.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline --no-stream-peak --no-refresh --no-parity > $out/bench_c${c}_q8.log 2>&1 || exit 1
done
for f in $out/bench_c*.log; do echo "$f"; grep -h '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['host'], d.get('parity') and d['parity']['mismatched_entries'])"; done
