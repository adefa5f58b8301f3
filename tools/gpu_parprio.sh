#!/bin/bash
# PAR slices' dispatch starts and wave times (CDR_PAR_PROF variants, with and without
# s_setprio 3 on the PAR waves), then the step time of each library in its own process
set -o pipefail
out=gpurun_out/${1:-ppr}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4 5}; do
  for v in prof profp3; do
    timeout -k 10 300 python3 -u tools/par_prof.py variants/libcdr_$v.so --config $c --top 4 > $out/${v}_c$c.log 2>&1 || { tail -20 $out/${v}_c$c.log; exit 1; }
    echo "$v C$c $(grep '^{' $out/${v}_c$c.log | cut -c1-900)"
  done
  for lib in cadence_amd/libcdr.so variants/libcdr_p3.so; do
    timeout -k 10 200 python3 -u tools/perf.py --config $c --rounds 2 --reps 5 $lib > $out/perf_c${c}_$(basename $lib .so).log 2>&1 || exit 1
    echo "C$c $lib $(grep median_ms $out/perf_c${c}_$(basename $lib .so).log | cut -c1-120)"
  done
done
