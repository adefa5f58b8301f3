#!/bin/bash
# Round 5, set H: class-kernel pending rows (A/T/X, reset points) written by the wave together — parity / full-size /
# class-kernel GPU tests, then interleaved A/B on C3 and C5
# (one library per process: multi-stream configs).
set -o pipefail
out=gpurun_out/${1:-r5h}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_cls_gpu.py tests/test_fullsize_gpu.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for c in 3 5; do
  for rep in 1 2; do
    for lib in variants/libcdr_g.so cadence_amd/libcdr.so; do
      n=$(basename $lib .so)
      timeout -k 10 200 python3 tools/perf.py --config $c --rounds 2 --reps 3 $lib > $out/c${c}_${n}_$rep.json 2>$out/c${c}_${n}_$rep.err || exit 1
      echo "C$c $n $rep $(tail -1 $out/c${c}_${n}_$rep.json | cut -c1-70)" >> $out/ab_c35.log
    done
  done
done
echo done
