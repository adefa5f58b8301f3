#!/bin/bash
# Round 5, set M: PAR / long-history planning knobs re-swept on the current kernels (C4, C5;
# one process per setting: the plan is made in-process from the env).
set -o pipefail
out=gpurun_out/${1:-r5m}; mkdir -p $out
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 200 python3 tools/perf.py --config $c --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}_$n.json 2>$out/c${c}_$n.err || exit 1
  echo "C$c $n $(tail -1 $out/c${c}_$n.json | cut -c1-80)" >> $out/sweep.log
}
for c in 4 5; do
  run base $c X=0
  run pm192 $c CDR_PAR_MAX=192
  run pm256 $c CDR_PAR_MAX=256
  run div4 $c CDR_LONG=1024,2,4,1
  run pm256div4 $c CDR_PAR_MAX=256 CDR_LONG=1024,2,4,1
  run pm384div4 $c CDR_PAR_MAX=384 CDR_LONG=1024,2,4,1
done
echo done
