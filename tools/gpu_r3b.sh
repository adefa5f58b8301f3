#!/bin/bash
# round 3: GPU suite, then C4/C5 stream-layout A/B (3 side streams, two groupings; 7 at 8 queues)
set -o pipefail
tag=${1:-r3b}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -60 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
B="--no-cpu-baseline --no-stream-peak --no-refresh --no-parity"
for c in 4 5 3; do
  timeout -k 10 400 python -u bench.py --config $c $B > $out/c${c}_g0555556.log 2>&1 || exit 1
  CDR_SIDE_GROUPS=0005556 timeout -k 10 400 python -u bench.py --config $c $B > $out/c${c}_g0005556.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u bench.py --config $c $B > $out/c${c}_q8.log 2>&1 || exit 1
done
for f in $out/c*.log; do echo "$f $(grep -h '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["roofline"]["kernel_ms"],3))')"; done
