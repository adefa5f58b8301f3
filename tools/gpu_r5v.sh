#!/bin/bash
# Round 5, set V: k_tasks_merge with the W list four records deep (libcdr.so) vs three (m3):
# task tests, then C3 / C5 --tasks, one library per process.
set -o pipefail
out=gpurun_out/${1:-r5v}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_tasks.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 5; do
  for rep in 1 2; do
    for lib in variants/libcdr_m3.so cadence_amd/libcdr.so; do
      n=$(basename $lib .so)
      timeout -k 10 200 python3 tools/perf.py --config $c --tasks --tasks-par --rounds 2 --reps 3 $lib > $out/c${c}_${n}_$rep.json 2>$out/c${c}_${n}_$rep.err || exit 1
      echo "C$c $n $rep $(tail -n 1 $out/c${c}_${n}_$rep.json | cut -c1-70)" >> $out/ab.log
    done
  done
done
echo done
