#!/bin/bash
# parity (incl. fast-path tests) + smoke + bench with and without the fast path
set -o pipefail
tag=${1:-fast}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/${tag}_parity.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream-peak > gpurun_out/${tag}_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream-peak --no-fast-path > gpurun_out/${tag}_bench_general.log 2>&1
rc=$?
echo "EXIT $rc"
tail -3 gpurun_out/${tag}_parity.log
tail -1 gpurun_out/${tag}_smoke.log 2>/dev/null
for f in gpurun_out/${tag}_bench.log gpurun_out/${tag}_bench_general.log; do
  grep "fast-path" $f 2>/dev/null
  grep -v "^\[rank\|amdgpu.ids" $f 2>/dev/null | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.rstrip()); continue
    r=d['roofline']; print('value %.4g ev/s  kernel_ms %.3f  achieved %.1f GB/s frac %.4f' % (d['value'], r['kernel_ms'], r['achieved'], r['frac']))
"
done
exit $rc
