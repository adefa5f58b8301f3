#!/bin/bash
# the GPU test suite (optionally a subset: tools/gpu_tests.sh OUT tests/x.py ...)
set -o pipefail
out=gpurun_out/${1:-t}; shift; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -30 $out/gpu_tests.log
exit $rc
