#!/bin/bash
# Round 5 final set, part 3 (same build): the configs[4] conflict-resolution line and the
# carry-in lines (with and without task lists), parity checked in each run.
set -o pipefail
out=gpurun_out/${1:-r5x}; mkdir -p $out
sha1sum cadence_amd/libcdr.so > $out/lib_sha1
timeout -k 10 600 python -u bench.py --ndc-forks --steps 5 --warmup 1 > $out/ndc_forks_1m.json 2> $out/ndc_forks_1m.log || exit 1
timeout -k 10 420 python -u bench.py --carry --config 5 --steps 10 --warmup 2 > $out/carry_c5.json 2> $out/carry_c5.log || exit 1
timeout -k 10 420 python -u bench.py --carry --tasks --config 3 --steps 10 --warmup 2 > $out/carry_tasks_c3.json 2> $out/carry_tasks_c3.log || exit 1
echo "extra set done"
