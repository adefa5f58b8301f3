#!/bin/bash
# --tasks lines with the plain lane plan (no wave / PAR slices): every register-table slice on
# the class kernels' TASKS instantiations; rocprofv3 kernel trace of the same command
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
for c in 5 3; do
  timeout -k 10 400 python3 -u bench.py --config $c --tasks --no-wave --no-par --steps 5 --warmup 2 --no-cpu-baseline --no-refresh --no-host-path --no-stream-peak > $out/c$c.json 2> $out/c$c.log || { tail $out/c$c.log; exit 1; }
  tail -c 300 $out/c$c.json; echo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/k$c -o run -- python3 bench.py --config $c --tasks --no-wave --no-par --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-refresh --no-host-path --no-stream-peak > $out/k$c.json 2> $out/k$c.log || exit 1
done
