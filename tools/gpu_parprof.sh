#!/bin/bash
# PAR per-wave loop times (variant -DCDR_PAR_PROF) and kernel timelines of C3-C5 at the
# default stream grouping
set -o pipefail
out=gpurun_out/${1:-pp}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  timeout -k 10 300 python3 -u tools/par_prof.py variants/libcdr_prof.so --config $c > $out/prof_c$c.log 2>&1 || { tail -20 $out/prof_c$c.log; exit 1; }
  grep '^{' $out/prof_c$c.log | cut -c1-1500
done
for c in ${TRACE:-3 4 5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/c${c}_q4 -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 cadence_amd/libcdr.so > $out/c${c}_q4.log 2>&1 || exit 1
  grep median $out/c${c}_q4.log
done
python3 tools/kernel_timeline.py $out > $out/timeline.txt 2>&1; cat $out/timeline.txt
