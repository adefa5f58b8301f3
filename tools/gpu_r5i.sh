#!/bin/bash
# Round 5, set I: the fast kernel's task records in one wave-wide LDS pool (record = its own
# destination; flush when the wave's records fill the pool) — task / carry GPU tests, then
# the C2 --tasks A/B in one process: the previous build (g) and pool sizes 5 / 8 / 12 x 64.
set -o pipefail
out=gpurun_out/${1:-r5i}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_tasks.py tests/test_carry.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/perf.py --config 2 --tasks --rounds 4 --reps 3 variants/libcdr_g.so variants/libcdr_t5.so cadence_amd/libcdr.so variants/libcdr_t12.so > $out/ab_t2.log 2>&1 || exit 1
echo done
