#!/bin/bash
# C3-C5 1M: long register-table histories on wave slices vs PAR slices (four-wave class kernel)
set -o pipefail
out=gpurun_out/${1:-parab}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5 3}; do
  for m in wave par; do
    flag=""; [ $m = wave ] && flag="--no-par"
    timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 $flag cadence_amd/libcdr.so > $out/c${c}_$m.json 2>$out/c${c}_$m.err || exit 1
    echo "C$c $m $(tail -1 $out/c${c}_$m.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_c4 -o run -- \
    python3 tools/perf.py --config 4 --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/trace_c4.log 2>&1
