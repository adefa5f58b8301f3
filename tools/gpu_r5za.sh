#!/bin/bash
# Round 5, set ZA: the epilogue flag fix with the flag held as a u32 instead of a bool,
# run through the carry tests and the class/newrun tests.
set -o pipefail
out=gpurun_out/${1:-r5za}; mkdir -p $out
CDR_LIB=variants/libcdr_${V:-epiint}.so timeout -k 10 300 python -u -m pytest tests/test_carry.py tests/test_cls_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $out/${V:-epiint}.log 2>&1; echo "rc=$?" >> $out/${V:-epiint}.log
echo done
