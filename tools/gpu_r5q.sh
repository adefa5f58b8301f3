#!/bin/bash
# Round 5, set Q: class-kernel tasks — merge before the retry pass, 3-deep merge prefetch;
# staging pool 4 x 64 (libcdr.so) vs 2 x 64 (ct2) vs 2 x 64 at 4 waves per SIMD (ct2w4);
# C3 / C5 --tasks with the PAR plan, one library per process; kernel trace of C3.
set -o pipefail
out=gpurun_out/${1:-r5q}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tasks.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 5; do
  for lib in cadence_amd/libcdr.so variants/libcdr_ct2.so variants/libcdr_ct2w4.so; do
    n=$(basename $lib .so)
    timeout -k 10 200 python3 tools/perf.py --config $c --tasks --tasks-par --rounds 2 --reps 3 $lib > $out/c${c}t_$n.json 2>$out/c${c}t_$n.err || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/tr_c3 -o run -- python3 tools/perf.py --config 3 --tasks --tasks-par --rounds 1 --reps 2 cadence_amd/libcdr.so > $out/tr_c3.log 2>&1 || exit 1
echo done
