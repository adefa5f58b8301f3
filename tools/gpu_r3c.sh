#!/bin/bash
# round 3 measurement set at HEAD: GPU suite, default C2 line (CPU baseline, parity),
# rocprofv3 kernel stats of the C2 bench, C3-C5 lines.  usage: tools/gpu_r3c.sh <tag>
set -o pipefail
tag=${1:-r3c}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -60 $out/gpu_tests.log; exit 1; }
  tail -3 $out/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > $out/bench_c2.log 2>&1 || { tail -30 $out/bench_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-stream-peak --no-parity > $out/trace.log 2>&1 || { tail -30 $out/trace.log; exit 1; }
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c > $out/bench_c$c.log 2>&1 || { tail -30 $out/bench_c$c.log; exit 1; }
done
for f in $out/bench_c*.log; do grep -h '^{' $f | cut -c1-400; done
