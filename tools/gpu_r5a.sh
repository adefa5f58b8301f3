#!/bin/bash
# Round 5, set A: the carry-in + tasks GPU tests, the 1M carry lines with task lists
# (C3, C5) and without, each step under its own limit; the chain stops at the first failure.
# usage: tools/gpu_r5a.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r5a}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 400 python -u -m pytest tests/test_tasks.py tests/test_carry.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py --carry --tasks --config 3 --steps 10 --warmup 2 > $out/carry_tasks_c3.json 2> $out/carry_tasks_c3.log &&
timeout -k 10 420 python -u bench.py --carry --tasks --config 5 --steps 10 --warmup 2 > $out/carry_tasks_c5.json 2> $out/carry_tasks_c5.log &&
timeout -k 10 420 python -u bench.py --carry --config 5 --steps 10 --warmup 2 > $out/carry_c5.json 2> $out/carry_c5.log
rc=$?
echo "r5a rc=$rc"
exit $rc
