#!/bin/bash
# --tasks lines (full-population digest parity + the sample's task-list parity) and the task tests
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tasks.py tests/test_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for c in 5 4 3; do
  timeout -k 10 400 python3 -u bench.py --config $c --tasks --steps 10 --warmup 2 --no-cpu-baseline --no-refresh --no-host-path --no-stream-peak > $out/c$c.json 2> $out/c$c.log || { tail $out/c$c.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/c$c.json').read().strip().splitlines()[-1]); print('C$c', round(d['ms_per_step'],3), d['parity_checked'], d['parity']['mismatched_entries'], d['parity']['tasks']['mismatched_entries'])"
done
