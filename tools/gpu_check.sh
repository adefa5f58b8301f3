#!/bin/bash
# One GPU round trip: parity + golden tests, smoke, bench (C2 1M).  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/${tag}_parity.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/${tag}_bench.log 2>&1
rc=$?
echo "EXIT $rc"
tail -2 gpurun_out/${tag}_parity.log
cat gpurun_out/${tag}_smoke.log 2>/dev/null | tail -1
grep -v "^\[rank\|amdgpu.ids" gpurun_out/${tag}_bench.log 2>/dev/null | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.rstrip()); continue
    r=d['roofline']; print('value %.4g ev/s  wf/s %.4g  ms/step %.3f  kernel_ms %.3f  achieved %.1f GB/s frac %.4f' % (d['value'], d['workflows_per_s'], d['ms_per_step'], r['kernel_ms'], r['achieved'], r['frac']))
"
exit $rc
