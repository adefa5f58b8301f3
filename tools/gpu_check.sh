#!/bin/bash
# all GPU tests, then per-kernel time split of one replay on configs 3,4,5 (1M workflows)
set -o pipefail
out=gpurun_out/${1:-chk}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c$c -o run -- \
    python3 tools/perf.py --config $c --wfs 1000000 --rounds 2 --reps 2 cadence_amd/libcdr.so > $out/c$c.log 2>&1 || exit 1
done
for c in ${CONFIGS:-3 4 5}; do echo "== C$c"; grep -h '^{' $out/c$c.log; find $out/c$c -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | head -7; done
