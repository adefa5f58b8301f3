#!/bin/bash
# bench lines + rocprofv3 kernel stats of configs 3-5 (class-decomposed register slices)
set -o pipefail
out=gpurun_out/${1:-bcls}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c > $out/bench_c$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_c$c -o run -- \
      python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-stream-peak --no-parity --no-refresh > $out/trace_c$c.log 2>&1 || exit 1
done
for c in ${CONFIGS:-3 4 5}; do grep -h '^{' $out/bench_c$c.log | cut -c1-400; done
