#!/bin/bash
# C5 --tasks: the PAR slices' histories one per slice (CDR_PAR_SOLO / CDR_PAR_MAX knobs), so
# that k_replay_reg<TASKS> steps one lane's handler group per row instead of sixteen lanes' union
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
f="--config 5 --tasks --steps 5 --warmup 2 --no-cpu-baseline --no-refresh --no-host-path --no-stream-peak --no-parity"
i=0
for e in "X=0" "CDR_PAR_SOLO=2048" "CDR_PAR_SOLO=256 CDR_PAR_MAX=16" "CDR_PAR_SOLO=512 CDR_PAR_MAX=32" "CDR_PAR_SOLO=1024 CDR_PAR_MAX=64"; do
  i=$((i+1))
  env $e timeout -k 10 300 python3 -u bench.py $f > $out/e$i.json 2> $out/e$i.log || { tail $out/e$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/e$i.json').read().strip().splitlines()[-1]); print('$e', round(d['ms_per_step'],3))"
done
