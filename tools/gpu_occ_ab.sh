#!/bin/bash
# class-kernel occupancy variants (waves/SIMD the register allocator targets) on C3 / C5
set -o pipefail
out=gpurun_out/${1:-occ}; mkdir -p $out
export TMPDIR=/tmp
for c in 3 5; do
  timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 cadence_amd/libcdr.so variants/libcdr_w5.so variants/libcdr_w5b.so variants/libcdr_w3.so > $out/c$c.json 2>$out/c$c.err || exit 1
  cat $out/c$c.json
done
