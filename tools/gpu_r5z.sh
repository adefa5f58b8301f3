#!/bin/bash
# Round 5, set Z: the register-table carry-path discrepancy — the carry tests on (a) the
# library with an unrelated no-op added to the register-table epilogue (allocation probe),
# (b) the epilogue flag fix, with carried entries on their own variants (CDR_CARRY_REG2=0),
# (c) the epilogue flag fix, default routing.
set -o pipefail
out=gpurun_out/${1:-r5z}; mkdir -p $out
t() { timeout -k 10 200 python -u -m pytest tests/test_carry.py -m gpu -q --timeout 120 --timeout-method thread "$@"; }
CDR_LIB=variants/libcdr_perturb.so t > $out/perturb.log 2>&1; echo "rc=$?" >> $out/perturb.log
CDR_LIB=variants/libcdr_epi3.so CDR_CARRY_REG2=0 t > $out/epi3_reg2off.log 2>&1; echo "rc=$?" >> $out/epi3_reg2off.log
CDR_LIB=variants/libcdr_epi3.so t > $out/epi3.log 2>&1; echo "rc=$?" >> $out/epi3.log
echo done
