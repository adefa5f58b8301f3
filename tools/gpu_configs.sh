#!/bin/bash
# C3-C5 bench lines (1M workflows per GPU), default routing and lane slices only.
set -o pipefail
tag=${1:-cfg}
mkdir -p gpurun_out
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-stream-peak \
      > gpurun_out/${tag}_c${c}.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-stream-peak --no-wave \
      > gpurun_out/${tag}_c${c}_lanes.log 2>&1 || exit $?
done
for f in gpurun_out/${tag}_c*.log; do
  echo "$f $(grep '^{' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("%.3g ev/s kernel %.2f ms frac %.4f" % (d["value"], r["kernel_ms"], r["frac"]))')"
done
