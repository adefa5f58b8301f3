#!/bin/bash
# Round 5, set K: the register-table kernels' task records in a wave-wide LDS pool — task /
# carry / parity GPU tests, then C3 --tasks A/B, one library per process (multi-stream config):
# reg pool off (r0), 3 / 4 (libcdr.so) / 6 x 64 records.
set -o pipefail
out=gpurun_out/${1:-r5k}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_tasks.py tests/test_carry.py tests/test_parity_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in variants/libcdr_r0.so variants/libcdr_r3.so cadence_amd/libcdr.so variants/libcdr_r6.so; do
    n=$(basename $lib .so)
    timeout -k 10 300 python3 tools/perf.py --config 3 --tasks --rounds 2 --reps 3 $lib > $out/c3t_${n}_$rep.json 2>$out/c3t_${n}_$rep.err || exit 1
    echo "C3t $n $rep $(tail -1 $out/c3t_${n}_$rep.json | cut -c1-90)" >> $out/ab.log
  done
done
echo done
