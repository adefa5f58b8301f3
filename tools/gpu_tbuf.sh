#!/bin/bash
# The fast kernel's TASKS instantiation with its LDS task buffer at 2/4/5/8 slots per lane
# (variants built with tools/build_variant.sh tbuf<N> -DCDR_FAST_TBUF=<N>): the task parity
# tests on two of them, then C2 --tasks step times against the in-tree build, twice each.
set -o pipefail
out=gpurun_out/tb; mkdir -p $out
for v in tbuf4 tbuf8; do
  CDR_LIB=variants/libcdr_$v.so timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tasks.py -m gpu > $out/t_$v.log 2>&1 || exit 1
done
for r in 1 2; do
  for v in base tbuf2 tbuf4 tbuf5 tbuf8; do
    if [ $v = base ]; then L=cadence_amd/libcdr.so; else L=variants/libcdr_$v.so; fi
    CDR_LIB=$L timeout -k 10 200 python bench.py --config 2 --tasks --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh > $out/c2_${v}_$r.json 2> $out/c2_${v}_$r.log || exit 1
  done
done
