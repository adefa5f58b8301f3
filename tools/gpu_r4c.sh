#!/bin/bash
# NDC GPU tests (incl. the 1M digests), 1M carry lines (C3, C5), NDC line PMC passes
set -o pipefail
out=gpurun_out/${1:-r4c}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ndc_gpu.py -m gpu > $out/ndc_tests.log 2>&1 || { tail -30 $out/ndc_tests.log; exit 1; }
tail -1 $out/ndc_tests.log
tools/gpu_carry.sh ${1:-r4c}/carry 3 1000000 && tools/gpu_carry.sh ${1:-r4c}/carry 5 1000000 && tools/gpu_ndc_pmc.sh r4ndc 1000000
