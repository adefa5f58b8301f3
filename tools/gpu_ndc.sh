#!/bin/bash
# configs[4] conflict-resolution line (bench.py --ndc-forks) and the NDC GPU tests
set -o pipefail
out=gpurun_out/${1:-ndc}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ndc_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 900 python -u bench.py --ndc-forks --wfs ${WFS:-100000} --steps 5 --warmup 1 > $out/ndc.log 2>&1 || { tail -30 $out/ndc.log; exit 1; }
grep -v '^{' $out/ndc.log | tail -5; grep '^{' $out/ndc.log | cut -c1-1500
