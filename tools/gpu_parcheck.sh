#!/bin/bash
# PAR kernel span in the trace vs its slices' own times (same run), and PAR slices alone
set -o pipefail
out=gpurun_out/${1:-pc}; mkdir -p $out
export TMPDIR=/tmp
for c in ${CONFIGS:-4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/prof_c$c -o run -- \
      python3 tools/par_prof.py variants/libcdr_prof.so --config $c --top 2 > $out/prof_c$c.log 2>&1 || { tail -20 $out/prof_c$c.log; exit 1; }
  grep '^{' $out/prof_c$c.log | cut -c1-400
  python3 - $out/prof_c$c/run_kernel_trace.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'replay' in r['Kernel_Name']]
t0 = min(int(r['Start_Timestamp']) for r in rows[-12:])
for r in rows[-12:]:
    print(r['Kernel_Name'][:48], r['Queue_Id'], (int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - t0) / 1e3)
PY
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/alone_c$c -o run -- \
      python3 tools/perf.py --config $c --rounds 1 --reps 3 --par-subset 128 cadence_amd/libcdr.so > $out/alone_c$c.log 2>&1 || exit 1
  grep median $out/alone_c$c.log
done
