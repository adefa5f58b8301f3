#!/bin/bash
# Round 5, set D: task emission with the loop-invariant task fields in registers — task tests,
# then the C2 and C3 --tasks lines (task lists checked against the oracle in the run).
set -o pipefail
out=gpurun_out/${1:-r5d}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 300 python -u -m pytest tests/test_tasks.py tests/test_carry.py -m gpu -x -v --timeout 90 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py --tasks --steps 10 --warmup 2 --no-refresh > $out/c2_tasks.json 2> $out/c2_tasks.log &&
timeout -k 10 420 python -u bench.py --tasks --config 3 --steps 10 --warmup 2 --no-refresh > $out/c3_tasks.json 2> $out/c3_tasks.log
rc=$?; echo "r5d rc=$rc"; exit $rc
