#!/bin/bash
# Round 5, set C: the fast kernel's task records written by the wave together — the task
# GPU tests, then the C2 --tasks line (task lists checked against the oracle in the run).
set -o pipefail
out=gpurun_out/${1:-r5c}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 300 python -u -m pytest tests/test_tasks.py -m gpu -x -v --timeout 90 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py --tasks --steps 10 --warmup 2 --no-refresh > $out/c2_tasks.json 2> $out/c2_tasks.log
rc=$?; echo "r5c rc=$rc"; exit $rc
