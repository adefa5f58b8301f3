#!/bin/bash
# parity + smoke + A/B of variant libraries + PMC passes of the main library
# usage: tools/gpu_ab.sh <tag> <variant.so>...   (env PERF_ARGS: extra tools/perf.py args)
set -o pipefail
tag=${1:-ab}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/${tag}_parity.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/perf.py $PERF_ARGS cadence_amd/libcdr.so "$@" > gpurun_out/${tag}_perf.log 2>&1 &&
bash tools/pmc.sh ${tag}
rc=$?
echo "EXIT $rc"
tail -2 gpurun_out/${tag}_parity.log
tail -1 gpurun_out/${tag}_smoke.log 2>/dev/null
grep -v "amdgpu.ids" gpurun_out/${tag}_perf.log 2>/dev/null | tail -6
exit $rc
