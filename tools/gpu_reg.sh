#!/bin/bash
# register-table kernel: parity then timing on C3/C4/C5 (1M workflows), reg on vs off
set -o pipefail
out=gpurun_out/${1:-reg}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $out/parity.log 2>&1 || { echo "parity failed"; tail -30 $out/parity.log; exit 1; }
for c in 3 4 5; do
  timeout -k 10 200 python tools/perf.py --config $c --wfs 1000000 --rounds 3 --reps 3 cadence_amd/libcdr.so > $out/c${c}_reg.log 2>&1 || exit 1
  timeout -k 10 200 python tools/perf.py --config $c --wfs 1000000 --rounds 2 --reps 2 --no-reg cadence_amd/libcdr.so > $out/c${c}_noreg.log 2>&1 || exit 1
done
grep -h '^{' $out/c*_*.log
