#!/bin/bash
# Round 5, set R: the class kernels' retry passes after the join (not beside the class kernels)
# — parity / class / full-size / task GPU tests, then A/B on C3 / C4 / C5 against the previous
# placement (g), one library per process, and C3 / C5 --tasks.
set -o pipefail
out=gpurun_out/${1:-r5r}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_cls_gpu.py tests/test_fullsize_gpu.py tests/test_tasks.py tests/test_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 4 5; do
  for rep in 1 2; do
    for lib in variants/libcdr_g.so cadence_amd/libcdr.so; do
      n=$(basename $lib .so)
      timeout -k 10 200 python3 tools/perf.py --config $c --rounds 2 --reps 3 $lib > $out/c${c}_${n}_$rep.json 2>$out/c${c}_${n}_$rep.err || exit 1
      echo "C$c $n $rep $(tail -n 1 $out/c${c}_${n}_$rep.json | cut -c1-70)" >> $out/ab.log
    done
  done
done
for c in 3 5; do
  timeout -k 10 200 python3 tools/perf.py --config $c --tasks --tasks-par --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}t.json 2>$out/c${c}t.err || exit 1
done
echo done
