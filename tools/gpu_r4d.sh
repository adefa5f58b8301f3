#!/bin/bash
# task + parity GPU tests, then the long-history A/B (tools/gpu_long_ab.sh); a crash, abort
# or timeout of the tests (rc other than 0 / 1) stops the call there
set -o pipefail
out=gpurun_out/${1:-r4d}; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tasks.py tests/test_parity_gpu.py -m gpu > $out/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $out/tests.log; tail -2 $out/tests.log
[ $rc -le 1 ] || exit $rc
tools/gpu_long_ab.sh ${2:-r4_lab}
