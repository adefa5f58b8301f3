#!/bin/bash
# issue-priority experiments: PAR slices (--par) with and without s_setprio; wave slices with s_setprio by length
set -o pipefail
out=gpurun_out/${1:-prio}; mkdir -p $out
export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 --par variants/libcdr_par_p0.so variants/libcdr_par_p3.so > $out/c${c}_par.json 2>$out/c${c}_par.err || exit 1
  cat $out/c${c}_par.json
  timeout -k 10 300 python3 tools/perf.py --config $c --rounds 3 --reps 3 variants/libcdr_par_p3.so variants/libcdr_wprio2k.so variants/libcdr_wprio1k.so > $out/c${c}_wave.json 2>$out/c${c}_wave.err || exit 1
  cat $out/c${c}_wave.json
done
