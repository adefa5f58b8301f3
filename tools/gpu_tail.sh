#!/bin/bash
# C2 fast-kernel time vs population: exactly 5 rounds of 3,072 resident slices (983,040 workflows) vs 1M (5.09 rounds)
set -o pipefail
out=gpurun_out/${1:-tail}; mkdir -p $out
export TMPDIR=/tmp
for n in 983040 1000000 1179648 1200000; do
  timeout -k 10 300 python3 tools/perf.py --config 2 --wfs $n --rounds 3 --reps 5 cadence_amd/libcdr.so > $out/n$n.json 2>$out/n$n.err || exit 1
  echo $n $(tail -1 $out/n$n.json)
done
