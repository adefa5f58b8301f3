#!/bin/bash
# Round 5, set O: where C3 --tasks time goes — the plan without PAR / wave slices (no tasks),
# --tasks with the PAR plan, and a kernel trace of each --tasks step.
set -o pipefail
out=gpurun_out/${1:-r5o}; mkdir -p $out
export TMPDIR=/tmp
for c in 3 5; do
  timeout -k 10 240 python3 tools/perf.py --config $c --no-wave --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}_plan0.json 2>$out/c${c}_plan0.err || exit 1
  timeout -k 10 240 python3 tools/perf.py --config $c --tasks --tasks-par --rounds 2 --reps 3 cadence_amd/libcdr.so > $out/c${c}t_par.json 2>$out/c${c}t_par.err || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace -d $out/tr_c$c -o run -- python3 tools/perf.py --config $c --tasks --rounds 1 --reps 2 cadence_amd/libcdr.so > $out/tr_c$c.log 2>&1 || exit 1
done
echo done
